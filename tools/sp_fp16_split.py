"""Where does fp16 SuperPoint lose keypoints?  A CPU emulation of the fp16 MFMA path (item 2 of the round-5
verdict): every layer chosen to be "fp16" takes its input activations and weights rounded to fp16, computes
in fp32 (an fp16 x fp16 product is exact in fp32, so this is the MFMA's arithmetic up to the accumulation
order) and, when the NEXT layer is fp16 too, its output is stored rounded to fp16 -- exactly the roundings of
librspl's fp16 kernels (sp_kernels.hip: conv3x3_h_kernel / conv1_res_kernel / det_head_h_kernel /
sample_taps_h_kernel).  An fp32 layer is the parity path's arithmetic.  The post-processing (NMS, threshold,
borders, top-k, fp64 sampling) is the oracle's (oracle/post.py), i.e. the reference's.

For each split it reports, over the C1 images (tools/run_c1_plumbing.py's synthetic.stereo_pair seeds
300..), the keypoint-set overlap with the fp32 oracle per image (mean / min), the fraction of identical sets,
the descriptor cosine on shared keypoints, and (--sg) the end-to-end match agreement through the oracle's fp32
SuperGlue with the c1 weight profile (the record's definition: |CPU ∩ fp16| / |CPU ∪ fp16| of the thresholded
matches by keypoint coordinates).  Test infrastructure: imports the oracle.
Usage: python tools/sp_fp16_split.py [--pairs 100] [--sg] [--splits all,enc16_head32,...]
"""
import argparse
import json
import pathlib
import sys

import numpy as np
import torch
import torch.nn.functional as Fn

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
import oracle  # noqa: E402
import post  # noqa: E402

H, W, K = 480, 752, 400
ENC = ["conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b"]
HEADS = ["convPa", "convPb", "convDa", "convDb"]
SPLITS = {
    "fp16_all": set(ENC + HEADS),                       # the product's fp16 path today
    "fp32_all": set(),
    "heads32": set(ENC),                                 # fp16 encoder, fp32 heads
    "det32": set(ENC + ["convDa", "convDb"]),            # fp32 detector head (convPa, convPb)
    "detb32": set(ENC + ["convPa", "convDa", "convDb"]),  # fp32 convPb only
    "conv1_32": set(ENC[2:] + HEADS),                    # fp32 conv1a / conv1b
    "conv4_32": set(ENC[:6] + HEADS),                    # fp32 conv4a / conv4b
    "late32": set(ENC[:6] + ["convDa", "convDb"]),       # fp32 conv4 + detector head
    "x3_all": {n: "x3" for n in ENC + HEADS},             # split fp16 everywhere (3 MFMA products)
    "x2a_all": {n: "x2a" for n in ENC + HEADS},           # activations split only
    "x2w_all": {n: "x2w" for n in ENC + HEADS},           # weights split only
    "x3_enc16c1": {**{n: "x3" for n in ENC[2:] + HEADS}, "conv1a": "16", "conv1b": "16"},  # conv1 fp16, rest split
}


def r16(t):
    return t.half().float()


def split16(t):
    """t = hi + lo, both fp16 (lo unscaled: it goes subnormal below |t| ~ 0.125, where its absolute error
    stays under fp16's subnormal spacing of 6e-8)"""
    hi = r16(t)
    return hi, r16(t - hi)


class Emu:
    """Per layer one of: "16" (fp16 operands, fp32 accumulation), "x3" (split fp16: activations and weights as
    hi + lo fp16 pairs, three MFMA products hi*hi + lo*hi + hi*lo accumulated in fp32), "x2a" / "x2w" (only the
    activations / only the weights split: two products), anything else fp32.  A layer's output is stored fp16
    only when the next layer is "16" (x2w too reads fp16 activations); otherwise it stays fp32 (x3 / x2a split
    it at load)."""
    def __init__(self, blob):
        self.w = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in pkg.weights.read_blob(blob).items()}

    def conv(self, x, name, mode, out16, relu=True, pad=1):
        w, b = self.w[name + ".weight"], self.w[name + ".bias"]
        if mode in ("16", "x2w"):
            x = r16(x)
        if mode == "16" and name == "conv1a":  # conv1_res_kernel: the bias rides the MFMA as the tenth tap (fp16)
            b = r16(b)
        if mode == "16":
            y = Fn.conv2d(x, r16(w), b, padding=pad)
        elif mode in ("x3", "x2a", "x2w"):
            xh, xl = split16(x)
            wh, wl = split16(w)
            y = Fn.conv2d(xh, wh, b, padding=pad)
            if mode in ("x3", "x2a"):
                y = y + Fn.conv2d(xl, wh, None, padding=pad)
            if mode in ("x3", "x2w"):
                y = y + Fn.conv2d(xh, wl, None, padding=pad)
        else:
            y = Fn.conv2d(x, w, b, padding=pad)
        if relu:
            y = Fn.relu(y)
        return r16(y) if out16 else y

    def forward(self, img_u8, half):
        """half: a set of fp16 layers, or a dict layer -> mode"""
        md = half if isinstance(half, dict) else {n: "16" for n in half}
        m = lambda n: md.get(n, "32")  # noqa: E731
        o16 = lambda n: m(n) in ("16", "x2w")  # noqa: E731  (the layer reads fp16 activations)
        x = torch.from_numpy(post.image_to_input(img_u8))[None, None]
        seq = ENC + ["convPa"]
        for i, name in enumerate(ENC):
            nxt = seq[i + 1]
            x = self.conv(x, name, m(name), m(name) != "32" and o16(nxt))
            if name in ("conv1b", "conv2b", "conv3b"):
                x = Fn.max_pool2d(x, 2, 2)
        pa = self.conv(x, "convPa", m("convPa"), m("convPa") != "32" and o16("convPb"))
        da = self.conv(x, "convDa", m("convDa"), m("convDa") != "32" and o16("convDb"))
        semi = self.conv(pa, "convPb", m("convPb"), False, relu=False, pad=0)
        desc = self.conv(da, "convDb", m("convDb"), False, relu=False, pad=0)
        s = torch.softmax(semi, 1)[:, :-1]
        h8, w8 = s.shape[2], s.shape[3]
        s = s.permute(0, 2, 3, 1).reshape(1, h8, w8, 8, 8).permute(0, 1, 3, 2, 4).reshape(h8 * 8, w8 * 8)
        desc = Fn.normalize(desc, p=2, dim=1)[0]
        scores = oracle.simple_nms(s.numpy().astype(np.float32))
        return post.sp_postprocess(scores, desc.numpy(), 0.004, 4, K)


def keys(F):
    return {(int(x), int(y)): i for i, (x, y) in enumerate(zip(F[1], F[2]))}


def coords(m, F0, F1):
    return {(int(F0[1, q]), int(F0[2, q]), int(F1[1, t]), int(F1[2, t])) for q, t in m}


def sg_matches(sg_w, F0, F1):
    G0, G1 = post.normalize_keypoints(F0, W, H), post.normalize_keypoints(F1, W, H)
    Z = oracle.sg_forward(sg_w, *post.sg_inputs(G0), *post.sg_inputs(G1))
    out = []
    for th in (0.0, 0.2):  # mutual nearest neighbours (the record's match_agreement), thresholded decode
        i0 = post.decode(Z, th)[0]
        out.append(coords([(q, int(t)) for q, t in enumerate(i0) if t >= 0], F0, F1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100)
    ap.add_argument("--sg", action="store_true")
    ap.add_argument("--splits", default=",".join(SPLITS))
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    oracle.set_threads(a.threads)
    sp_w, _ = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    sg_w = pkg.weights.ensure_sg_profile_blob(str(ROOT / "weights"), "c1")
    emu = Emu(sp_w)
    names = a.splits.split(",")
    stats = {n: {"overlap": [], "cos": [], "agree": [], "agree_th": []} for n in names}
    for t in range(a.pairs):
        L, R = pkg.synthetic.stereo_pair(H, W, seed=300 + t)
        ref = [emu.forward(im, SPLITS["fp32_all"]) for im in (L, R)]
        mref = sg_matches(sg_w, *ref) if a.sg else None
        for n in names:
            F = ref if n == "fp32_all" else [emu.forward(im, SPLITS[n]) for im in (L, R)]
            for Fr, Fe in zip(ref, F):
                kr, ke = keys(Fr), keys(Fe)
                sh = set(kr) & set(ke)
                stats[n]["overlap"].append(len(sh) / max(1, len(kr)))
                if sh:
                    dr = np.array([Fr[3:, kr[c]] for c in sh])
                    de = np.array([Fe[3:, ke[c]] for c in sh])
                    stats[n]["cos"].append(float(np.min(np.sum(dr * de, 1))))
            if a.sg:
                me = sg_matches(sg_w, *F)
                stats[n]["agree"].append(len(mref[0] & me[0]) / max(1, len(mref[0] | me[0])))
                stats[n]["agree_th"].append(len(mref[1] & me[1]) / max(1, len(mref[1] | me[1])))
        if t % 10 == 9:
            print(f"pair {t + 1}: " + ", ".join(f"{n} ovl min {min(stats[n]['overlap']):.4f}" for n in names),
                  file=sys.stderr, flush=True)
    out = {}
    for n in names:
        s = stats[n]
        out[n] = {"layers": SPLITS[n] if isinstance(SPLITS[n], dict) else {k: "16" for k in sorted(SPLITS[n])},
                  "images": len(s["overlap"]),
                  "keypoint_overlap_mean": float(np.mean(s["overlap"])), "keypoint_overlap_min": float(np.min(s["overlap"])),
                  "keypoint_sets_identical_frac": float(np.mean([o == 1.0 for o in s["overlap"]])),
                  "desc_cos_min": float(np.min(s["cos"])) if s["cos"] else None}
        if a.sg:
            out[n]["match_agreement_mean"] = float(np.mean(s["agree"]))
            out[n]["match_agreement_min"] = float(np.min(s["agree"]))
            out[n]["thresholded_agreement_mean"] = float(np.mean(s["agree_th"]))
            out[n]["thresholded_agreement_min"] = float(np.min(s["agree_th"]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
