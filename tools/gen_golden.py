"""Generate the committed golden fixtures under tests/golden/ (runs ONLY in the
build container, where /root/reference is mounted).

Outputs are produced by the reference's own PyTorch model definitions
(convert2onnx/superpoint.py, convert2onnx/superglue.py -- imported from the
reference tree, never copied) with deterministic synthetic weights
(rspl-slam_amd/weights.py), plus the numpy restatement of the reference's
host C++ (oracle/post.py) for threshold/top-k/sampling/decode/matching.

Usage:  python tools/gen_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import hashlib
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
from rspl_slam_amd import weights as W  # noqa: E402
from rspl_slam_amd import synthetic as SY  # noqa: E402
import post  # noqa: E402  (oracle/post.py)

OUT = ROOT / "tests" / "golden"


def load_reference(ref: str):
    sys.path.insert(0, str(pathlib.Path(ref) / "convert2onnx"))
    import torch
    import superpoint  # reference module
    import superglue   # reference module
    torch.set_num_threads(8)
    sp = superpoint.SuperPoint().eval()
    sp.load_state_dict({k: torch.from_numpy(v) for k, v in W.superpoint_synth(1).items()})
    sg = superglue.SuperGlue().eval()
    sg.load_state_dict({k: torch.from_numpy(v) for k, v in W.superglue_synth(2).items()}, strict=False)
    return torch, superpoint, superglue, sp, sg


def run_sp(torch, sp, img):
    x = torch.from_numpy(post.image_to_input(img))[None, None]
    with torch.no_grad():
        s, d = sp(x)
    return s[0].numpy(), d[0].numpy()


def run_sg(torch, sg, F0, F1, width, height):
    G0 = post.normalize_keypoints(F0, width, height)
    G1 = post.normalize_keypoints(F1, width, height)
    k0, s0, d0 = post.sg_inputs(G0)
    k1, s1, d1 = post.sg_inputs(G1)
    T = torch.from_numpy
    with torch.no_grad():
        Z = sg(T(k0)[None], T(s0)[None], T(d0)[None], T(k1)[None], T(s1)[None], T(d1)[None])
    return Z[0].numpy()


def gen_sg_c1(torch, superglue, sp):
    """C1 stereo pair (synthetic.stereo_pair seed 300, 480x752, k = 400) through the reference modules:
    SuperPoint (seeded weights) on both images + the host post-processing restatement, then SuperGlue with
    the "c1" weight profile (weights.SG_WEIGHT_GAIN_C1: matches above the 0.2 threshold), decode and
    PointMatching's DMatches.  Features are rounded to float32 (SuperGlue::process_input packs floats)."""
    sgc = superglue.SuperGlue().eval()
    sgc.load_state_dict({k: torch.from_numpy(v) for k, v in W.superglue_synth(2, "c1").items()}, strict=False)
    L, R = SY.stereo_pair(480, 752, seed=300)
    F = []
    for img in (L, R):
        s, d = run_sp(torch, sp, img)
        F.append(post.sp_postprocess(s, d, 0.004, 4, 400).astype(np.float32).astype(np.float64))
    Z = run_sg(torch, sgc, F[0], F[1], 752, 480)
    idx0, idx1, ms0, ms1 = post.decode(Z)
    mt, md = post.match_points(idx0, idx1, ms0, ms1)
    np.savez_compressed(OUT / "sg_c1.npz", seed=300, F0=F[0].astype(np.float32), F1=F[1].astype(np.float32),
                        width=752, height=480, Z=Z, idx0=idx0, idx1=idx1, ms0=ms0, ms1=ms1, matches=mt,
                        distances=md)
    print("sg_c1", Z.shape, "matches", len(mt))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="generate one fixture only (sg_c1)")
    args = ap.parse_args()
    OUT.mkdir(parents=True, exist_ok=True)
    torch, superpoint, superglue, sp, sg = load_reference(args.ref)
    if args.only == "sg_c1":
        gen_sg_c1(torch, superglue, sp)
        return

    # 1. SP-small: 64x96, k=32 -----------------------------------------------------------
    img = SY.textured_image(64, 96, seed=1, n_blobs=8)
    s, d = run_sp(torch, sp, img)
    F = post.sp_postprocess(s, d, 0.004, 4, 32)
    np.savez_compressed(OUT / "sp_small.npz", image=img, scores=s, desc=d, features=F,
                        threshold=0.004, border=4, k=32)
    print("sp_small", F.shape)

    # 2. SP-EuRoC: 480x752, k=400 -----------------------------------------------------
    img = SY.textured_image(480, 752, seed=0)
    s, d = run_sp(torch, sp, img)
    F = post.sp_postprocess(s, d, 0.004, 4, 400)
    nz = np.nonzero(s.reshape(-1))[0]
    rng = np.random.default_rng(7)
    samp = rng.integers(0, d.size, size=4096)
    np.savez_compressed(OUT / "sp_euroc.npz", image=img,
                        feat_head=F[:3], feat_desc=F[3:].astype(np.float32),
                        nms_idx=nz.astype(np.int32), nms_val=s.reshape(-1)[nz],
                        desc_sample_idx=samp.astype(np.int64), desc_sample_val=d.reshape(-1)[samp],
                        scores_sha256=np.frombuffer(hashlib.sha256(s.tobytes()).digest(), np.uint8),
                        threshold=0.004, border=4, k=400)
    print("sp_euroc", F.shape, "nms nonzero", nz.size)

    # 3. NMS unit: random maps and a plateau map with exact ties -------------------
    rng = np.random.default_rng(3)
    maps = [rng.random((40, 56)).astype(np.float32),
            (rng.random((33, 47)) ** 4).astype(np.float32)]
    plateau = np.zeros((40, 48), np.float32)
    plateau[5:12, 5:12] = 0.5                    # flat plateau: all equal
    plateau[20, 20] = 0.7
    plateau[22, 23] = 0.7                        # two equal peaks inside one window
    plateau[30:33, 30:40] = np.linspace(0.1, 0.3, 10, dtype=np.float32)
    maps.append(plateau)
    outs = []
    for m in maps:
        with torch.no_grad():
            outs.append(superpoint.simple_nms(torch.from_numpy(m)[None], 4)[0].numpy())
    np.savez_compressed(OUT / "nms_unit.npz", **{f"in{i}": m for i, m in enumerate(maps)},
                        **{f"out{i}": o for i, o in enumerate(outs)})
    print("nms_unit", len(maps))

    # 4. Sinkhorn + decode unit ------------------------------------------------------------
    rng = np.random.default_rng(4)
    sc = (rng.normal(size=(1, 64, 56)) * 3).astype(np.float32)
    alpha = torch.tensor(1.0)
    with torch.no_grad():
        Zs = superglue.log_optimal_transport(torch.from_numpy(sc), alpha, 100)[0].numpy()
    dec = post.decode(Zs)
    # decode tie case: duplicated maxima in row 3 / column 5
    Zt = Zs.copy()
    Zt[3, 10] = Zt[3, :-1].max()
    Zt[7, 5] = Zt[:-1, 5].max()
    dect = post.decode(Zt)
    np.savez_compressed(OUT / "sinkhorn_unit.npz", scores=sc[0], alpha=1.0, iters=100, Z=Zs,
                        idx0=dec[0], idx1=dec[1], ms0=dec[2], ms1=dec[3],
                        Z_ties=Zt, t_idx0=dect[0], t_idx1=dect[1], t_ms0=dect[2], t_ms1=dect[3])
    print("sinkhorn_unit", Zs.shape, "valid", (dec[0] >= 0).sum())

    # 5. SG-small: N=48, M=40 (full chain, matches) -----------------------------
    F0, F1, gt = SY.sg_problem(48, 40, 30, seed=5)
    Z = run_sg(torch, sg, F0, F1, 752, 480)
    idx0, idx1, ms0, ms1 = post.decode(Z)
    mt, md = post.match_points(idx0, idx1, ms0, ms1)
    np.savez_compressed(OUT / "sg_small.npz", F0=F0, F1=F1, gt=gt, width=752, height=480, Z=Z,
                        idx0=idx0, idx1=idx1, ms0=ms0, ms1=ms1, matches=mt, distances=md)
    print("sg_small", Z.shape, "matches", len(mt))

    # 6. SG-400: N=400, M=380 ---------------------------------------------------------------
    F0, F1, gt = SY.sg_problem(400, 380, 300, seed=6)
    F0 = F0.astype(np.float32).astype(np.float64)   # stored as float32 below: keep inputs exact
    F1 = F1.astype(np.float32).astype(np.float64)
    Z = run_sg(torch, sg, F0, F1, 752, 480)
    idx0, idx1, ms0, ms1 = post.decode(Z)
    mt, md = post.match_points(idx0, idx1, ms0, ms1)
    np.savez_compressed(OUT / "sg_400.npz", F0=F0.astype(np.float32), F1=F1.astype(np.float32), gt=gt,
                        width=752, height=480, Z=Z, idx0=idx0, idx1=idx1, ms0=ms0, ms1=ms1,
                        matches=mt, distances=md)
    print("sg_400", Z.shape, "matches", len(mt))

    # 7. weight-generator pin: first values of a few tensors --------------------------------
    spw = W.superpoint_synth(1)
    sgw = W.superglue_synth(2)
    pins = {k: spw[k].reshape(-1)[:16] for k in ["conv1a.weight", "convPb.weight", "convDb.bias"]}
    pins.update({k: sgw[k].reshape(-1)[:16] for k in ["kenc.encoder.0.weight", "kenc.encoder.1.running_var",
                                                     "gnn.layers.17.mlp.3.weight", "final_proj.weight"]})
    np.savez_compressed(OUT / "weights_pin.npz", **{k.replace(".", "__"): v for k, v in pins.items()})
    print("weights_pin")

    # 8. C1 stereo pair with the "c1" SuperGlue profile -------------------------------------
    gen_sg_c1(torch, superglue, sp)


if __name__ == "__main__":
    main()
