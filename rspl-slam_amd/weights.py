"""Deterministic synthetic weights and the RSPLWT01 weight-blob format.

No pretrained SuperPoint / SuperGlue weights exist in this environment
(SURVEY.md F1), so every parity test runs on synthetic weights produced by
the generator below.  The generator is counter-based and uses only IEEE
operations that are correctly rounded (integer mixing, one sqrt, multiplies,
adds), so numpy here and any C/C++ restatement produce bit-identical float32
tensors.

Tensor names and shapes are exactly the reference state_dict keys:
  SuperPoint  -- convert2onnx/superpoint.py:86-105
  SuperGlue   -- convert2onnx/superglue.py:51-85,126-173,244-259
so a real ``superpoint_v1.pth`` / ``superglue_indoor.pth`` state_dict can be
converted to the same blob (tools/convert_weights.py) and loaded unchanged.

Generator spec (per tensor ``name``, global ``seed``):
  base   = splitmix64_mix(seed ^ fnv1a64(name))
  u_i    = (splitmix64_mix(base + (i+1)*0x9E3779B97F4A7C15) >> 11) * 2**-53   in [0,1)
  value  = lo + (hi - lo) * u_i      (computed in float64, rounded once to float32)
with (lo, hi) from ``_range_for`` (He-uniform for conv weights, documented
small ranges for biases / BatchNorm statistics).

Blob layout (little endian):
  b"RSPLWT01" | u32 count | count x { u32 name_len | name | u32 ndim |
  i64 dims[ndim] | f32 data[prod(dims)] }
"""
from __future__ import annotations

import math
import struct
from collections import OrderedDict

import numpy as np

MAGIC = b"RSPLWT01"
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """n float64 values in [0,1) for tensor ``name`` (exact, platform independent)."""
    base = _mix(np.uint64((seed ^ fnv1a64(name)) & 0xFFFFFFFFFFFFFFFF))
    idx = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _mix(base + idx * _GAMMA)
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


# --------------------------------------------------------------------------
# canonical tensor lists (reference state_dict order)
# --------------------------------------------------------------------------
def superpoint_shapes() -> "OrderedDict[str, tuple]":
    """convert2onnx/superpoint.py:88-105"""
    c1, c2, c3, c4, c5 = 64, 64, 128, 128, 256
    convs = [("conv1a", 1, c1, 3), ("conv1b", c1, c1, 3), ("conv2a", c1, c2, 3),
             ("conv2b", c2, c2, 3), ("conv3a", c2, c3, 3), ("conv3b", c3, c3, 3),
             ("conv4a", c3, c4, 3), ("conv4b", c4, c4, 3), ("convPa", c4, c5, 3),
             ("convPb", c5, 65, 1), ("convDa", c4, c5, 3), ("convDb", c5, 256, 1)]
    d = OrderedDict()
    for name, cin, cout, k in convs:
        d[f"{name}.weight"] = (cout, cin, k, k)
        d[f"{name}.bias"] = (cout,)
    return d


def _bn(d, prefix, c):
    d[f"{prefix}.weight"] = (c,)
    d[f"{prefix}.bias"] = (c,)
    d[f"{prefix}.running_mean"] = (c,)
    d[f"{prefix}.running_var"] = (c,)


def superglue_shapes(n_layers: int = 18) -> "OrderedDict[str, tuple]":
    """convert2onnx/superglue.py:51-85 (kenc), 126-173 (gnn), 254-259 (final_proj, bin_score)"""
    d = OrderedDict()
    d["bin_score"] = ()
    chans = [3, 32, 64, 128, 256, 256]
    for i in range(1, len(chans)):
        li = 3 * (i - 1)
        d[f"kenc.encoder.{li}.weight"] = (chans[i], chans[i - 1], 1)
        d[f"kenc.encoder.{li}.bias"] = (chans[i],)
        if i < len(chans) - 1:
            _bn(d, f"kenc.encoder.{li + 1}", chans[i])
    for l in range(n_layers):
        p = f"gnn.layers.{l}"
        d[f"{p}.attn.merge.weight"] = (256, 256, 1)
        d[f"{p}.attn.merge.bias"] = (256,)
        for j in range(3):
            d[f"{p}.attn.proj.{j}.weight"] = (256, 256, 1)
            d[f"{p}.attn.proj.{j}.bias"] = (256,)
        d[f"{p}.mlp.0.weight"] = (512, 512, 1)
        d[f"{p}.mlp.0.bias"] = (512,)
        _bn(d, f"{p}.mlp.1", 512)
        d[f"{p}.mlp.3.weight"] = (256, 512, 1)
        d[f"{p}.mlp.3.bias"] = (256,)
    d["final_proj.weight"] = (256, 256, 1)
    d["final_proj.bias"] = (256,)
    return d


# Synthetic-weight profile.  Scales chosen (and measured) so
# that (a) SuperPoint scores are distinct (reference top-k uses a non-stable
# std::sort) and (b) SuperGlue descriptors keep their identity
# through 18 residual layers so synthetic matching problems have real
# mutual matches above the 0.2 threshold.
SP_WEIGHT_GAIN = {"convPb.weight": 4.0}
SG_WEIGHT_GAIN = {"kenc.encoder.12.weight": 0.05, "mlp.3.weight": 0.1, "final_proj.weight": 8.0}
# "c1" SuperGlue profile (same seed and generator, other gains): a 6x stronger keypoint-encoder output and
# a 2x final projection sharpen the assignment so that on the C1 stereo pairs (SuperPoint features of
# synthetic.stereo_pair, seeded SuperPoint weights) 25-38 % of the keypoints are matched above the
# reference's 0.2 threshold (super_glue.cpp:355; measured on seeds 300-305 through the oracle: 100-154
# matches per pair of 400, median row gap of the matched log-assignments 0.5) -- the default profile keeps
# every probability below 0.2 there, so the thresholded decode and the DMatch distances were never
# exercised on SuperPoint-derived features.
SG_WEIGHT_GAIN_C1 = {"kenc.encoder.12.weight": 0.3, "mlp.3.weight": 0.1, "final_proj.weight": 16.0}
SG_PROFILES = {"default": SG_WEIGHT_GAIN, "c1": SG_WEIGHT_GAIN_C1}
BIAS_RANGE = 0.05


def _range_for(name: str, shape: tuple, gains: dict):
    if name.endswith("running_mean"):
        return -0.1, 0.1
    if name.endswith("running_var"):
        return 0.5, 1.5
    is_bn = (".running" not in name) and len(shape) == 1 and _is_bn_param(name)
    if is_bn and name.endswith(".weight"):
        return 0.5, 1.5
    if is_bn and name.endswith(".bias"):
        return -0.1, 0.1
    if name == "bin_score":
        return None
    if name.endswith(".bias"):
        return -BIAS_RANGE, BIAS_RANGE
    fan_in = int(np.prod(shape[1:]))
    a = math.sqrt(6.0 / fan_in)
    g = 1.0
    for suffix, gain in gains.items():
        if name.endswith(suffix):
            g = gain
    return -a * g, a * g


def _is_bn_param(name: str) -> bool:
    # BatchNorm layers live at kenc.encoder.{1,4,7,10} and gnn.layers.*.mlp.1
    parts = name.split(".")
    if parts[0] == "kenc":
        return int(parts[2]) % 3 == 1
    if parts[0] == "gnn":
        return parts[-3] == "mlp" and parts[-2] == "1"
    return False


def synth(shapes: "OrderedDict[str, tuple]", seed: int, gains: dict) -> "OrderedDict[str, np.ndarray]":
    out = OrderedDict()
    for name, shape in shapes.items():
        n = int(np.prod(shape)) if shape else 1
        rng = _range_for(name, shape, gains)
        if rng is None:  # bin_score: reference init torch.tensor(1.)
            arr = np.array(1.0, dtype=np.float32)
        else:
            lo, hi = rng
            u = uniform01(seed, name, n)
            arr = (lo + (hi - lo) * u).astype(np.float32).reshape(shape)
        out[name] = arr
    return out


def superpoint_synth(seed: int = 1) -> "OrderedDict[str, np.ndarray]":
    return synth(superpoint_shapes(), seed, SP_WEIGHT_GAIN)


def superglue_synth(seed: int = 2, profile: str = "default") -> "OrderedDict[str, np.ndarray]":
    return synth(superglue_shapes(), seed, SG_PROFILES[profile])


# --------------------------------------------------------------------------
# blob I/O
# --------------------------------------------------------------------------
def write_blob(path, tensors: "OrderedDict[str, np.ndarray]") -> None:
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<I", len(tensors)))
        for name, arr in tensors.items():
            a = np.ascontiguousarray(arr, dtype="<f4")
            nb = name.encode()
            f.write(struct.pack("<I", len(nb)))
            f.write(nb)
            f.write(struct.pack("<I", a.ndim))
            for s in a.shape:
                f.write(struct.pack("<q", s))
            f.write(a.tobytes())


def read_blob(path) -> "OrderedDict[str, np.ndarray]":
    out = OrderedDict()
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != MAGIC:
        raise ValueError(f"{path}: not an RSPLWT01 blob")
    off = 8
    (count,) = struct.unpack_from("<I", data, off)
    off += 4
    for _ in range(count):
        (nl,) = struct.unpack_from("<I", data, off)
        off += 4
        name = data[off:off + nl].decode()
        off += nl
        (nd,) = struct.unpack_from("<I", data, off)
        off += 4
        dims = struct.unpack_from("<" + "q" * nd, data, off)
        off += 8 * nd
        n = int(np.prod(dims)) if nd else 1
        arr = np.frombuffer(data, dtype="<f4", count=n, offset=off).reshape(dims).copy()
        off += 4 * n
        out[name] = arr
    return out


def ensure_blobs(directory, sp_seed: int = 1, sg_seed: int = 2):
    """Write weights/superpoint_synth_s{seed}.bin and superglue_synth_s{seed}.bin if absent."""
    import os
    os.makedirs(directory, exist_ok=True)
    sp = os.path.join(directory, f"superpoint_synth_s{sp_seed}.bin")
    sg = os.path.join(directory, f"superglue_synth_s{sg_seed}.bin")
    if not os.path.exists(sp):
        write_blob(sp, superpoint_synth(sp_seed))
    if not os.path.exists(sg):
        write_blob(sg, superglue_synth(sg_seed))
    return sp, sg


def ensure_sg_profile_blob(directory, profile: str = "c1", sg_seed: int = 2):
    """weights/superglue_synth_s{seed}_{profile}.bin (written if absent)."""
    import os
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"superglue_synth_s{sg_seed}_{profile}.bin")
    if not os.path.exists(path):
        write_blob(path, superglue_synth(sg_seed, profile))
    return path
