#!/usr/bin/env python3
"""Headline benchmark: stereo frames/sec through SuperPoint -> SuperGlue -> local BA @ 752x480.

Workload (BASELINE.json configs[2], "C3", all-keyframe worst case of SURVEY.md §8d): every
step is one stereo keyframe of a synthetic EuRoC-shaped stream:
  * SuperPoint on the rectified stereo pair (batch 2, 480x752, top-400),
  * SuperGlue/PointMatching on 2 pairs: left(t) vs left(t-1) keyframe, left(t) vs right(t),
  * the line front end of the stereo keyframe: LineDetector::LineExtractor on both images' RCF-like edge
    maps (the restated FLD, rspl_lines_detect: GPU resize / Sobel / Canny classes, host chaining and
    fitting, then the host merge passes) on two native worker threads beside SuperPoint / SuperGlue, as the
    reference's line threads run beside its point thread (src/map_builder.cc:285-290, 325-337), joined
    before the line part of Frame::AddRightFeatures (src/frame.cc:150-203): both images'
    AssignPointsToLines, the stereo-match disparity filter and MatchLines on the GPU
    (rspl_lines_stereo_device), fed by SuperPoint's device features and SuperGlue's device match index of
    the left(t)-right(t) pair,
  * one local BA (LocalmapOptimization) of a C3-sized problem: 10 keyframes (1 fixed),
    ~4k points / ~10^4 point observations, 100 lines (synthetic, with ground truth).
Inputs (images) are resident in HBM before timing.  BA is host-driven and runs on its own
(highest-priority) stream, overlapping the frame's SP/SG exactly as the reference's tracking
thread overlaps its feature thread (src/map_builder.cc:48-49); SP of frame t+1 runs on its own
stream beside SG of frame t (event-ordered).  The timed region ends with a device
synchronisation, so every frame's SP, SG and BA work is inside it.  The BA problem is handed over as host
arrays (the reference's std::map containers), so its H2D upload is inside the step.

Multi-GPU: `bench.py --gpus N` spawns N rank processes itself (before anything touches the GPU),
or runs as one rank under `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
(then WORLD_SIZE must equal N).  One process per GPU; each rank runs its own stereo sequence
(replicas, weak scaling); a torch-free TCP host group (rspl-slam_amd/hostgroup.py) provides the barrier, the
max-over-ranks timing and the rank census (fails loudly if fewer than N distinct GPUs come up).  `--ba-mode shard` instead
solves every step's N local BAs (one per rank's sequence) jointly, landmark-sharded over all
ranks with an RCCL all-reduce of the reduced camera system per LM trial.

Workloads: `--workload c3` (default, BASELINE configs[2]), `c4` (configs[3]'s per-GPU sequence:
OIVIO-shaped 640x512 stereo, 600 keypoints, SG N=600; with --gpus 8 one sequence per GPU) or `c5`
(configs[4]: synthetic 1920x1080 stereo, 2048 keypoints, SG N=2048, 30-keyframe / 10k-landmark BA).
"""
import argparse
import gc
import json
import os
import queue
import threading
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# SP, SG and BA each need their own hardware queue to overlap (HIP maps streams round-robin
# onto GPU_MAX_HW_QUEUES queues; with the default 4 the SP and SG streams land on one queue
# and serialise).  Must be set before the HIP runtime initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
capi = pkg.capi

WORKLOADS = {
    "c3": dict(H=480, W=752, K=400, ba=dict(n_poses=10, n_points=4000, n_lines=100), ba_caps=(16, 6000, 200, 40000),
               desc="C3 EuRoC 752x480 stereo keyframe stream: SP batch 2 top-400, SG 2 pairs N=400, "
                    "local BA 10 poses / ~4k points / 100 lines"),
    "c4": dict(H=512, W=640, K=600, ba=dict(n_poses=10, n_points=4000, n_lines=100), ba_caps=(16, 6000, 200, 40000),
               desc="C4 OIVIO-shaped 640x512 stereo keyframe stream (one sequence per GPU): SP batch 2 top-600, SG 2 "
                    "pairs N=600, local BA 10 poses / ~4k points / 100 lines"),
    "c5": dict(H=1080, W=1920, K=2048, ba=dict(n_poses=30, n_points=10000, n_lines=0, pixel_sigma=0.8,
                                               outlier_frac=0.05), ba_caps=(32, 10000, 16, 70000),
               desc="C5 synthetic 1920x1080 stereo stream: SP batch 2 top-2048, SG 2 pairs N=2048, "
                    "local BA 30 keyframes / 10k landmarks (5 % outliers)"),
}
H, W, K = 480, 752, 400  # set from the workload in main()
FP32_MFMA_PEAK = 157.3  # TFLOP/s, MI355X_MICROARCH.md (v_mfma_f32_32x32x2_f32, dense)
FP16_MFMA_PEAK = 2516.8  # TFLOP/s dense (~2.5 PF, = 16 x the f32 MFMA rate), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0  # HBM3E, MI355X_MICROARCH.md


def conv1_gflop_per_image():
    return 2 * H * W * 64 * 9 / 1e9 + 2 * H * W * 64 * 576 / 1e9  # conv1a + conv1b


def ba_bytes_per_iteration(prob):
    """algorithmic bytes of one LM iteration = N_obs (4 d + 8) (measurements + ids)
    + 12 N_pt + 24 N_line + 28 K + 8 ((6K)^2 + 6K) (parameters, reduced-system write)."""
    sets = (("mono", 2), ("stereo", 3), ("mono_line", 4), ("stereo_line", 8))
    nobs = sum(d * prob.n_edges(n) for n, d in sets)
    nedges = sum(prob.n_edges(n) for n, _ in sets)
    Kp = int((prob.pose_fixed == 0).sum())
    return 4 * nobs + 8 * nedges + 12 * len(prob.points) + 24 * len(prob.lines) + 28 * Kp + \
        8 * ((6 * Kp) ** 2 + 6 * Kp)


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def cpu_baseline(sp_w, sg_w, frames, threads, wl):
    """The oracle's C restatement (oracle/*.c) of the same per-keyframe work on host cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # checker/baseline only
    import post
    oracle.set_threads(threads)
    syn = pkg.synthetic
    probs = [syn.ba_problem(seed=100 + i, **wl["ba"])[0] for i in range(frames)]
    pairs = [syn.stereo_pair(H, W, seed=200 + i) for i in range(frames + 1)]
    prev = None
    t0 = time.perf_counter()
    for f in range(frames):
        L, R = pairs[f]
        feats = []
        for img in (L, R):
            s, d = oracle.sp_forward(sp_w, post.image_to_input(img))
            feats.append(post.sp_postprocess(s, d, 0.004, 4, K))
        if prev is None:
            prev = feats[0]
        for a, b in ((feats[0], prev), (feats[0], feats[1])):
            ga, gb = post.normalize_keypoints(a, W, H), post.normalize_keypoints(b, W, H)
            Z = oracle.sg_forward(sg_w, *post.sg_inputs(ga), *post.sg_inputs(gb))
            post.decode(Z)
        oracle.ba_local(probs[f])
        prev = feats[0]
    dt = time.perf_counter() - t0
    return {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{frames} stereo keyframes (2xSP + 2xSG + 1 local BA each, same shapes) "
                      f"through the oracle's C restatement, OMP_NUM_THREADS={threads}, {dt:.1f} s"}


def _pmc_files(kind, workload):
    """Committed PMC summaries of `kind` ("traffic" / "mfma") for the workload, newest round first.
    C3 (the headline) files are profiles/rNN_pmc_<kind>_fp16.json; the side workloads carry their own
    passes as profiles/rNN_pmc_<kind>_fp16_<workload>.json -- a summary is never borrowed across configs."""
    files = sorted((ROOT / "profiles").glob(f"*_pmc_{kind}*.json"), reverse=True)
    if workload == "c3":
        return [f for f in files if not any(f.stem.endswith("_" + w) for w in WORKLOADS if w != "c3")]
    return [f for f in files if f.stem.endswith("_" + workload)]


def pmc_traffic(kernel_substr, workload="c3"):
    """HBM bytes per launch of a kernel from the newest committed PMC summary for this workload
    (profiles/*_pmc_traffic*.json, written by tools/pmc_traffic.py from two rocprofv3
    --pmc passes, FETCH_SIZE x2 gfx950 correction), or None."""
    for f in _pmc_files("traffic", workload):
        for name, v in json.loads(f.read_text()).items():
            if kernel_substr in name:
                return v["traffic_bytes"], f.name
    return None, None


def pmc_mfma(kernel_substr, workload="c3"):
    """MFMA-busy of a kernel from the newest committed rocprofv3 PMC pass for this workload
    (profiles/*_pmc_mfma*.json, tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x 1024
    SIMDs = rocprofv3's MfmaUtil, and over the busy CUs' SIMD cycles), or None."""
    for f in _pmc_files("mfma", workload):
        for name, v in json.loads(f.read_text()).items():
            if kernel_substr in name:
                return {"chip": round(v["mfma_busy_chip"], 4),
                        "per_busy_cu": round(v["mfma_busy_per_busy_cu"], 4) if v.get("mfma_busy_per_busy_cu") else None,
                        "source": f"profiles/{f.name}"}
    return None


def stage_roofline(sp, sg, sp_ms, sp_calls, sg_ms, sg_calls, precision, workload):
    """Achieved rate vs the bounding peak for the big stages (HIP-event stage times on the stage's
    launch stream, per step: 2 SuperPoint images, 2 SuperGlue pairs of N = M = K).  Algorithmic work
    as SURVEY.md 8(d): conv1a+conv1b 2*H*W*64*(9 + 576) FLOP per image; GNN 2*(655,360 N + 512 N M)
    per image per layer; Sinkhorn compulsory 2*4*(N+1)(M+1) bytes per pair (couplings in, Z out); NMS 4*H*W (the score
    map read once; the product path writes no NMS'd map, the candidates carry the scores)
    bytes per image.  Single-kernel stages carry the kernel name (pmc_kernel) whose PMC traffic
    summary under profiles/ gives `traffic`; the GNN is a launch family (single_kernel false)."""
    t = {**{f"sp:{n}": v / max(1, sp_calls) for n, v in zip(sp.STAGES, sp_ms)},
         **{f"sg:{n}": v / max(1, sg_calls) for n, v in zip(sg.STAGES, sg_ms)}}
    N = M = K
    h16 = precision in ("fp16", "fp16x3")  # fp16 MFMA operands (fp16x3: SuperPoint split into hi + lo)
    mfma_peak = FP16_MFMA_PEAK if h16 else FP32_MFMA_PEAK
    # the fused conv1a + conv1b + pool kernel of each precision (fp16: persistent, conv1b weights resident in LDS)
    conv1_k = {"fp16": "conv1_res_kernel", "fp16x3": "conv3x3_x3_kernel<64, 16, true, true>",
               "fp32": "conv3x3_kernel<64, 16, true, true>"}[precision]
    rows = (("sp:conv1a+1b+pool", 2 * conv1_gflop_per_image(), "TFLOP/s", mfma_peak, "mfma", conv1_k, True,
             "GFLOP per launch (2 images, conv1a+conv1b)"),
            ("sg:gnn x18", 2 * 2 * 18 * 2 * (655360 * N + 512 * N * M) / 1e9, "TFLOP/s", mfma_peak, "mfma",
             "layer_kernel" if h16 else "gemm_kernel", False,
             "GFLOP per step (2 pairs x 2 images x 18 layers; fp16: 19 launches of the fused layer kernel, "
             "fp32: 4 GEMM/attention launches per layer)"),
            ("sg:sinkhorn", 2 * 2 * 4 * (N + 1) * (M + 1) / 1e9, "GB/s", HBM_PEAK_GBS, "hbm",
             "sinkhorn_w_kernel" if N + 1 > 640 else "sinkhorn_sc_kernel",
             True, "GB per launch (2 pairs, compulsory: couplings read + Z written once, 2*4*(N+1)(M+1) per pair; "
                   "the kernel holds K = exp(C + a + b) in registers across the 100 iterations)"),
            ("sp:nms", 2 * 4 * H * W / 1e9, "GB/s", HBM_PEAK_GBS, "hbm", "nms_kernel", True,
             "GB per launch (2 images, 4*H*W: the score map read once)"))
    out = {}
    for key, work, unit, peak, bound, kern, single, what in rows:
        ms = t.get(key)
        if ms:
            ach = work / ms if unit == "TFLOP/s" else work / ms * 1e3
            nl = 19 if key == "sg:gnn x18" and h16 else 1  # launches per step of the kernel
            out[key] = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                        "frac": round(ach / peak, 4), "ms": round(ms, 4), "avg_launch_ms": round(ms / nl, 5),
                        "launches_per_step": nl, "algorithmic": f"{work:.4g} {what}", "pmc_kernel": kern,
                        "single_kernel": single or nl > 1}
    for r in out.values():
        if r["bound"] == "mfma":
            r["mfma_busy"] = pmc_mfma(r["pmc_kernel"], workload)
        tr, src = pmc_traffic(r["pmc_kernel"], workload)
        r["traffic"] = round(tr) if tr and r["single_kernel"] else None
    return out


def ba_kernel_rows(prob, kt, timed_calls, workload):
    """Roofline rows of the local BA's two per-trial launches from their HIP-event times on the BA stream
    (LocalBA.kernel_times over every call of the instrumented pass that follows the timed region).  Algorithmic bytes per launch =
    the records the launch must read once plus what it writes:
      Schur chunks + fused solve: per edge of an optimised pose Hpl (6 x ld) + Hpp (21) + bp (6), per
        landmark Hll (ld x ld) + bl (ld), doubles; the 48-double sums of each pose pair written, the
        reduced system read back by the solver and the 6K solution written;
      update: per edge the observation (2 / 3 / 4 / 8 doubles), its ids (16 B) and Hpl (6 x ld), the
        error (4) and robust cost written, the speculative records (Hpp 21 + bp 6 + Hpl 6 x ld) written;
        per landmark its state read and written and Hll / bl read and written."""
    names = ("mono", "stereo", "mono_line", "stereo_line")
    ne = {n: prob.n_edges(n) for n in names}
    npt, nln = len(prob.points), len(prob.lines)
    Kp = int((prob.pose_fixed == 0).sum())
    ld = {"mono": 3, "stereo": 3, "mono_line": 4, "stereo_line": 4}
    dobs = {"mono": 2, "stereo": 3, "mono_line": 4, "stereo_line": 8}
    rec = sum(ne[n] * (6 * ld[n] + 21 + 6) for n in names)
    lmk = npt * (9 + 3) + nln * (16 + 4)
    npairs = Kp * (Kp + 1) // 2
    chunk_b = 8 * (rec + lmk + npairs * 48 * 2 + 6 * Kp)
    upd_b = sum(ne[n] * (8 * (dobs[n] + 6 * ld[n] + 4 + 1 + 21 + 6 + 6 * ld[n]) + 16) for n in names) + \
        8 * (2 * (3 * npt + 6 * nln) + npt * (9 + 3) * 2 + nln * (16 + 4) * 2)
    rows = {}
    for key, (ms, n), b, kern, what in (
            ("ba:schur chunks+solve", kt["chunks+solve"], chunk_b, "pair_chunk_kernel",
             "records read once (Hpl, Hpp, bp per edge; Hll, bl per landmark) + pose-pair sums + solve I/O"),
            ("ba:update", kt["update"], upd_b, "update_errors_kernel",
             "observations, ids and Hpl read; errors, costs and the speculative records written")):
        if n:
            avg = ms / n
            rows[key] = {"bound": "hbm", "achieved": round(b / avg * 1e-6, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(b / avg * 1e-6 / HBM_PEAK_GBS, 5), "avg_launch_ms": round(avg, 5),
                         "ms": round(avg * n / max(1, timed_calls), 4), "launches_per_call": round(n / max(1, timed_calls), 2),
                         "algorithmic": f"{b / 1e6:.4g} MB per launch: {what}", "pmc_kernel": kern,
                         "single_kernel": True}
            tr, _ = pmc_traffic(kern, workload)
            rows[key]["traffic"] = round(tr) if tr else None
    return rows


def ate_report(ba):
    """'ATE vs ref' (BASELINE.json metric) at the trajectory level: a synthetic 20-keyframe stereo
    sequence (synthetic.map_sequence: tracked poses with drift, landmarks, 4 % gross outliers) goes
    keyframe by keyframe through the native Map -- Map::LocalMapOptimization with the GPU local BA
    (src/map.cc:537-808) -- and the keyframe trajectory (SaveKeyframeTrajectory, map.cc:1007-1024) is
    scored like run_batch.py:48 (evo_ape tum -a: association, SE(3) Umeyama, translation RMSE)
    against (a) the same sequence through the oracle's restatement of the map and of g2o, (b) ground
    truth; (c) the tracked (drifting) input poses against ground truth, for scale.  Also the map-side
    LocalMapOptimization time per keyframe (assembly + GPU BA + outliers + write-back)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # checker only
    import map_ref  # checker only
    from rspl_slam_amd import sequence as SQ, trajectory as TJ
    seq = pkg.synthetic.map_sequence(n_keyframes=20, n_points=3000, n_lines=40, seed=21, outlier_frac=0.04)
    t = time.perf_counter()
    m, reports = SQ.run(seq, ba)
    lmo_ms = (time.perf_counter() - t) * 1e3 / len(reports)
    mr = map_ref.Map(seq["camera"])
    for k, kf in enumerate(seq["keyframes"]):
        map_ref.insert_keyframe(mr, kf)
        if k:
            map_ref.local_map_optimization(mr, kf["id"], oracle.ba_local)
    ts = seq["timestamps"]
    P = np.array([m.GetPose(kf["id"])[:3, 3] for kf in seq["keyframes"]])
    P_o = np.array([mr.keyframes[kf["id"]].pose[:3, 3] for kf in seq["keyframes"]])
    gt = seq["gt_Twc"][:, :3, 3]
    tracked = np.array([kf["Twc"][:3, 3] for kf in seq["keyframes"]])
    return {"vs_reference_restatement_m": TJ.ape(ts, P_o, ts, P)["rmse"],
            "vs_ground_truth_m": TJ.ape(ts, gt, ts, P)["rmse"],
            "tracked_input_vs_ground_truth_m": TJ.ape(ts, gt, ts, tracked)["rmse"],
            "keyframes": len(ts), "point_outliers_removed": int(sum(r["n_point_outliers"] for r in reports)),
            "map_local_ba_ms_per_keyframe": round(lmo_ms, 3),
            "note": "trajectory ATE (evo_ape -a restatement) of a synthetic 20-keyframe sequence through the "
                    "native Map + GPU LocalMapOptimization; reference = oracle map + g2o restatement"}


def replica_seeds(rank):
    """Per-rank synthetic sequence (replicas: each GPU runs its own stereo stream)."""
    return {"images": [1000 * rank + i for i in range(4)], "ba": [1000 * rank + 50 + i for i in range(3)]}


def job_time(elapsed, group=None):
    """Whole-job wall time = max over ranks of each rank's timed region (host-group all-reduce)."""
    if group is None:
        return elapsed
    return group.allreduce_max(elapsed)


def job_value(world, steps, elapsed):
    """frames/s over all ranks: every rank processed `steps` stereo keyframes."""
    return world * steps / elapsed


def spawn_ranks(n, argv, script=None):
    """bench.py --gpus N without a launcher: start N rank processes (one per GPU) before this
    process touches the GPU, wait for all of them, exit with the first failure's code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script or pathlib.Path(__file__).resolve())] + argv, env=env))
    rc = 0
    while [pr.poll() for pr in procs].count(None):  # poll every rank each round
        bad = [pr.returncode for pr in procs if pr.returncode not in (None, 0)]
        if bad:  # one rank failed: the others would wait on it forever
            rc = bad[0]
            for q in procs:
                if q.poll() is None:
                    q.kill()
            break
        time.sleep(0.2)
    for pr in procs:
        pr.wait()
        if pr.returncode and not rc:
            rc = pr.returncode
    if rc:
        log(f"bench: a rank exited with {rc}")
    return rc


def rank_census(group, world, want, local, cnt):
    """Every rank reports (rank, device, visible devices, host); fail loudly unless exactly `want`
    ranks came up on distinct GPUs."""
    rows = group.all_gather([group.rank, local, cnt, os.uname().nodename])
    bad = [r for r in rows if r[1] >= r[2]]
    if bad:
        raise SystemExit(f"bench: ranks want GPUs that are not visible (rank, device, visible, host): {bad}")
    devs = {(h, d) for _, d, _, h in rows}
    if world != want or len(devs) != world:
        raise SystemExit(f"bench: --gpus {want} but {world} ranks on {len(devs)} distinct GPUs came up: {rows}")
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--ba-mode", choices=["replica", "shard"], default="replica",
                    help="replica: each rank solves its own sequence's BA; shard: every step's N BAs are solved "
                         "jointly, landmark-sharded over all ranks (RCCL all-reduce of the reduced camera system)")
    ap.add_argument("--cpu-frames", type=int, default=None, help="keyframes in the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ba-thread", choices=["native", "python"], default="native",
                    help="the tracking thread that runs the local BAs: the BA handle's native host thread "
                         "(rspl_ba_submit) or a Python thread around rspl_ba_local (A/B)")
    ap.add_argument("--precision", choices=["fp32", "fp16", "fp16x3"], default="fp16",
                    help="SP/SG MFMA precision: fp16x3 = SuperPoint in split fp16 (hi + lo operands, three fp16 MFMA "
                         "products: the fp32 path's keypoint sets) with SuperGlue in fp16; "
                         "fp16 = the reference's own TensorRT kFP16 engines "
                         "(src/super_point.cpp:98, src/super_glue.cpp:132; default), fp32 = the parity path")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="CUs the SuperPoint/SuperGlue streams leave free for the BA chain (CU-masked streams)")
    ap.add_argument("--ba-own-cus", type=int, default=1,
                    help="1: the BA runs only on the reserved CUs (disjoint from SP/SG)")
    ap.add_argument("--skip", default="", help="diagnostics only: comma list of stages to leave out (sp,sg,ba)")
    ap.add_argument("--ba-ktime-steps", type=int, default=20,
                    help="steps of the instrumented pass after the timed region whose BA calls time the BA's two "
                         "per-trial launches with HIP events (0: off); the timed region carries no BA events")
    ap.add_argument("--single-precision", action="store_true",
                    help="skip the second (other-precision) measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    global H, W, K
    wl = WORKLOADS[args.workload]
    H, W, K = wl["H"], wl["W"], wl["K"]
    capi.load()  # librspl's HIP runtime first: one runtime per process
    dist = None  # host group (barrier, max-over-ranks time, census, RCCL id): no torch in this process
    if world > 1:
        dist = pkg.hostgroup.HostGroup(rank, world, timeout=300.0)
        rank_census(dist, world, args.gpus, local, capi.device_count())
    capi.check(capi.load().rspl_set_device(local), "rspl_set_device")

    sp_w, sg_w = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    # the second measurement of the same run: the fp16 headline is paired with the split-fp16 SuperPoint (the
    # fp32 path's keypoint sets, profiles/r06_c1_plumbing.json), the others with fp16
    other_prec = {"fp16": "fp16x3", "fp16x3": "fp16", "fp32": "fp16"}
    precs = [args.precision] + ([other_prec[args.precision]] if world == 1 and not args.single_precision else [])
    handles = {}
    for pr in precs:  # all handles and streams created once, up front: fixed HW-queue placement
        code = capi.RSPL_PREC_FP16 if pr in ("fp16", "fp16x3") else capi.RSPL_PREC_FP32  # SuperGlue
        sp_code = capi.RSPL_PREC_FP16X3 if pr == "fp16x3" else code
        sp_h = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=K, weights=sp_w, max_height=H, max_width=W,
                                                   max_batch=2, precision=sp_code, device=local))
        assert sp_h.build(), sp_h.error
        sg_h = pkg.SuperGlue(pkg.SuperGlueConfig(image_width=W, image_height=H, weights=sg_w, max_keypoints=K,
                                                 max_batch=2, precision=code, device=local))
        assert sg_h.build(), sg_h.error
        handles[pr] = (sp_h, sg_h)
    ba = pkg.LocalBA(*wl["ba_caps"], device=local)
    if args.ba_own_cus and args.reserve_cus > 0:
        ba.use_reserved_cus(args.reserve_cus)
    shard = args.ba_mode == "shard"
    if shard:  # landmark-sharded BA over RCCL: one communicator across all ranks (also valid at N = 1)
        # librccl prints its version banner on stdout: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            uid = pkg.broadcast_comm_id(dist) if dist is not None else pkg.comm_unique_id()
            comm = pkg.Comm(uid, rank, world, local)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        ba.set_comm(comm)
    syn = pkg.synthetic
    NP = 4
    pool = capi.DeviceBuffer(NP * 2 * H * W)
    seeds = replica_seeds(rank)
    for i in range(NP):
        L, R = syn.stereo_pair(H, W, seed=seeds["images"][i])
        pool.upload(np.stack([L, R]), offset=i * 2 * H * W)
    if shard:  # every rank holds every rank's problems: step i solves all N of them jointly
        ba_sets = [syn.ba_problem(seed=sd, **wl["ba"]) for r in range(world) for sd in replica_seeds(r)["ba"]]
    else:
        ba_sets = [syn.ba_problem(seed=sd, **wl["ba"]) for sd in seeds["ba"]]
    problems = [p for p, _ in ba_sets]
    FB = K * 259 * 8
    # SP(t+1) is pipelined beside SG(t): SP and SG on their own streams,
    # ordered by events; feature slots triple-buffered (SG(t) reads slots t and t-1,
    # SP(t+1) writes slot t+1 and first waits for SG(t-1), the last reader of that slot)
    feats = [capi.DeviceBuffer(2 * FB) for _ in range(3)]
    counts = [capi.DeviceBuffer(8) for _ in range(3)]
    for c in counts:
        c.zero()
    f0, f1 = capi.DeviceBuffer(2 * FB), capi.DeviceBuffer(2 * FB)
    n0, n1 = capi.DeviceBuffer(8), capi.DeviceBuffer(8)
    outs = [capi.DeviceBuffer(2 * K * sz) for sz in (4, 4, 8, 8)]
    # SG is the frame's critical chain (SP has slack): SG and the BA run at high priority.  With
    # --reserve-cus the SP / SG / post streams are CU-masked off a few CUs spread over the chip
    # (and, with --ba-own-cus, the BA confined to them).  Measured: no gain -- the BA's slowdown
    # under load is memory-latency contention, not CU slots -- so the default is 0 (unmasked)
    rc = args.reserve_cus
    # stream priorities: SG and its post stream high (the BA's own stream is always high), SP normal
    prio = dict(sp="normal", sg="high", post="high")
    st_sp, st_sg = capi.Stream(reserve_cus=rc, priority=prio["sp"]), capi.Stream(reserve_cus=rc, priority=prio["sg"])
    st_post = capi.Stream(reserve_cus=rc, priority=prio["post"])  # SG's Sinkhorn + decode: overlaps the next GNN
    ev_sp = [capi.Event() for _ in range(3)]
    ev_sg = [capi.Event() for _ in range(3)]
    # line front end of each stereo keyframe: per replica frame a left / right RCF-like edge map in host
    # memory (the reference reads image_rcf from disk); every step runs LineDetector::LineExtractor on both
    # on two host threads (one detector handle each) and uploads the lines for the stereo association,
    # which runs on the post stream after the decode (frame.cc:150-203)
    lm = pkg.lines.LineMatcher(max_lines=512, max_points=max(K, 512), device=local)
    edge_imgs = [syn.edge_stereo_pair(H, W, seed=seeds["images"][i]) for i in range(NP)]
    # one detector handle per image, each with its native worker thread (rspl_lines_extract_async): the
    # feature thread only submits and joins, as the reference's line threads (no Python threads)
    detectors = [pkg.lines.LineDetector(device=local) for _ in range(2)]
    line_bufs = [(capi.DeviceBuffer(512 * 4 * 8), capi.DeviceBuffer(512 * 4 * 8)) for _ in range(3)]
    lines_out, lines_valid = capi.DeviceBuffer(512 * 4 * 8), capi.DeviceBuffer(512)
    line_stats = {"detect_ms": [], "lines": []}

    bf = pkg.synthetic.EUROC_BF
    cam_limits = (bf / 10.0, bf / 0.1, 2.0)  # MinXDiff, MaxXDiff, MaxYDiff (camera.cc:21-22, euroc.yaml)

    trace_path = os.environ.get("RSPL_BENCH_TRACE")  # diagnostics: per-step / per-BA-call host timeline
    trace_on = bool(trace_path)
    trace_out = []
    step_tr = []

    def measure(precision):
        """One full timed run of the pipeline at `precision`; returns its measurements."""
        sp, sg = handles[precision]
        for c in counts:
            c.zero()
        capi.synchronize()
        ba_ms = []
        ba_iters = []
        ba_err = []
        ba_q = queue.Queue(maxsize=2)

        def tracking_thread():
            """BA worker: the reference runs LocalmapOptimization on the tracking thread while the
            feature thread keeps extracting/matching (src/map_builder.cc:48-49, src/map.cc:105-107)."""
            capi.check(capi.load().rspl_set_device(local), "rspl_set_device")  # HIP device is per thread
            outs_ba = {}  # one result buffer per problem, reused (the bench reads only the counters)
            while True:
                item = ba_q.get()
                if item is None:
                    ba_q.task_done()
                    return
                t = time.perf_counter()
                try:
                    for prob in item:
                        r = ba.run(prob, out=outs_ba.get(id(prob)))
                        outs_ba[id(prob)] = r
                        ba_iters.append(r.iters_first + r.iters_second)
                except Exception as e:  # surfaced on the main thread
                    ba_err.append(e)
                ba_ms.append((time.perf_counter() - t) * 1e3 / len(item))
                ba_q.task_done()

        native = args.ba_thread == "native"
        if not native:
            worker = threading.Thread(target=tracking_thread, daemon=True)
            worker.start()
        outs_nat = {}  # native tracking thread: one result buffer per problem, reused

        def ba_put(item):
            """hand keyframe i's local BA to the tracking thread: the handle's native host thread
            (rspl_ba_submit: blocks while two calls wait, map_builder.cc:176), or the Python one (A/B)"""
            if not native:
                ba_q.put(item)
                return
            for prob in item:
                outs_nat[id(prob)] = ba.submit(prob, out=outs_nat.get(id(prob)))

        def ba_drain():
            if not native:
                ba_q.join()
                return
            n, its, ms = ba.join()
            if n:
                per = len(ba_item(0))
                ba_ms.extend([ms / n] * (n // per))
                ba_iters.extend([its / n] * (n // per))
        kt_steps = 0 if shard else args.ba_ktime_steps  # instrumented BA pass after the timed region
        line_timers = []  # HIP-event timers around the line association (post stream), timed steps only

        def ba_item(i):
            if shard:  # all ranks' BAs of step i, each solved jointly by every rank
                return [problems[(i % len(seeds["ba"])) + len(seeds["ba"]) * r] for r in range(world)]
            return [problems[i % len(problems)]]

        def step(i):
            if trace_on:  # host timeline of the step (RSPL_BENCH_TRACE): its start, then named marks
                step_tr.append({"i": i, "t": time.perf_counter()})
            slot, pslot = i % 3, (i - 1) % 3
            cur, prev, ccur, cprev = feats[slot], feats[pslot], counts[slot], counts[pslot]
            skip = args.skip.split(",")
            # the line threads of this keyframe, beside its SuperPoint / SuperGlue (map_builder.cc:325-337)
            eL, eR = edge_imgs[i % NP]
            jobs = None
            if "lines" not in skip:
                tw = time.perf_counter()
                detectors[0].submit(eL)
                detectors[1].submit(eR)
                jobs = detectors
                host_wait["line_submit"] += time.perf_counter() - tw
            if "sp" in skip or "sg" in skip:  # diagnostics: stages left out (not a benchmark line)
                if jobs is not None:
                    jobs[0].wait(), jobs[1].wait()
                if "sp" not in skip:
                    sp.infer_device(pool.offset((i % NP) * 2 * H * W), 2, H, W, W, H * W, cur.ptr, K, ccur.ptr,
                                    st_sp.handle)
                if "sg" not in skip:
                    sg.infer_device(2, f0.ptr, n0.ptr, f1.ptr, n1.ptr, K, True, outs[0].ptr, outs[1].ptr,
                                    outs[2].ptr, outs[3].ptr, st_sg.handle, post_stream=st_post.handle)
                if "ba" not in skip:
                    ba_put(ba_item(i))
                return
            tw = time.perf_counter()
            if i >= 2:
                ev_sg[(i - 2) % 3].wait_on(st_sp.handle)
            sp.infer_device(pool.offset((i % NP) * 2 * H * W), 2, H, W, W, H * W, cur.ptr, K, ccur.ptr, st_sp.handle)
            ev_sp[slot].record(st_sp.handle)
            host_wait["sp_calls"] += time.perf_counter() - tw
            tw = time.perf_counter()
            if trace_on:
                step_tr[-1]["sp"] = tw
            ev_sp[slot].wait_on(st_sg.handle)
            # PointMatching pairs: (L_t, L_kf) and (L_t, R_t)
            capi.memcpy_d2d(f0.ptr, cur.ptr, FB, st_sg.handle)
            capi.memcpy_d2d(f0.offset(FB), cur.ptr, FB, st_sg.handle)
            capi.memcpy_d2d(f1.ptr, prev.ptr, FB, st_sg.handle)
            capi.memcpy_d2d(f1.offset(FB), cur.offset(FB), FB, st_sg.handle)
            capi.memcpy_d2d(n0.ptr, ccur.ptr, 4, st_sg.handle)
            capi.memcpy_d2d(n0.offset(4), ccur.ptr, 4, st_sg.handle)
            capi.memcpy_d2d(n1.ptr, cprev.ptr, 4, st_sg.handle)
            capi.memcpy_d2d(n1.offset(4), ccur.offset(4), 4, st_sg.handle)
            sg.infer_device(2, f0.ptr, n0.ptr, f1.ptr, n1.ptr, K, True, outs[0].ptr, outs[1].ptr, outs[2].ptr,
                            outs[3].ptr, st_sg.handle, post_stream=st_post.handle)
            host_wait["sg_calls"] += time.perf_counter() - tw
            if trace_on:
                step_tr[-1]["sg"] = time.perf_counter()
            # stereo line association of frame t: the joined line threads' lines, SP's device records of
            # (left, right) and SG's match index of pair 1 (left(t) -> right(t)), stream-ordered behind the
            # decode
            if jobs is not None:
                # join the line workers; their lines go to the device in post-stream order (no host sync)
                tw = time.perf_counter()
                dl0, dl1 = line_bufs[slot]
                nl0, t0ms = jobs[0].wait_device(dl0.ptr, 512, st_post.handle)
                nl1, t1ms = jobs[1].wait_device(dl1.ptr, 512, st_post.handle)
                host_wait["lines"] += time.perf_counter() - tw
                if trace_on:
                    step_tr[-1]["lines"] = time.perf_counter()
                if line_t0 is not None:
                    line_stats["detect_ms"].append(max(t0ms, t1ms))
                    line_stats["lines"].append(nl0 + nl1)
                tw = time.perf_counter()
                tm = line_timers[i - line_t0] if line_t0 is not None else None
                if tm is not None:
                    tm.start(st_post.handle)
                lm.stereo_lines_device(dl0.ptr, nl0, dl1.ptr, nl1, cur.ptr, K, ccur.ptr, outs[0].offset(K * 4),
                                       cam_limits, lines_out.ptr, lines_valid.ptr, st_post.handle)
                if tm is not None:
                    tm.stop(st_post.handle)
                host_wait["line_assoc_calls"] += time.perf_counter() - tw
            ev_sg[slot].record(st_post.handle)  # matches and lines complete on the post stream
            # keyframe i's local BA goes to the tracking thread (own high-priority stream) through a
            # 2-deep buffer, as the reference's feature thread blocks only while
            # _tracking_data_buffer.size() >= 2 (src/map_builder.cc:176)
            if "ba" not in skip:
                tw = time.perf_counter()
                if trace_on:
                    step_tr[-1]["ba_put0"] = tw
                ba_put(ba_item(i))
                host_wait["ba_queue"] += time.perf_counter() - tw
                if trace_on:
                    step_tr[-1]["ba_put1"] = time.perf_counter()

        host_wait = {"lines": 0.0, "ba_queue": 0.0, "sp_calls": 0.0, "sg_calls": 0.0, "line_assoc_calls": 0.0,
                     "line_submit": 0.0}
        # the warmup steps run exactly the timed steps' code path, measurement included (stage timers, the
        # line-association timers), so no first-use cost lands in the timed region.  (The 7-10 ms stall of the
        # first timed BA calls that round 4's 20-step bench showed was the H2D hipMemcpyAsync, not this: fixed by
        # the upload kernel, profiles/r05_bench_20step.json.)  The BA's per-launch HIP events are NOT in the timed
        # region: they cost every timed call a host round trip (the final kernel is then host-ordered) and 45
        # event records (918 vs 883 frames/s on one box); they run in the instrumented pass after it.
        sp.profile(True)
        sg.profile(True)
        ba.kernel_timing(0)
        line_timers[:] = [capi.Timer() for _ in range(args.warmup)]
        line_t0 = 0
        # the cyclic garbage collector off for the warmup and the timed steps (as timeit does): a full
        # collection walks every object torch has created -- a multi-ms pause of the Python feature thread
        # that drains the pipeline (seen as single ~5-8 ms stalls in 20-step runs); reference counting still
        # frees each step's temporaries
        gc.collect()
        gc.freeze()
        gc.disable()
        for i in range(args.warmup):
            step(i)
        ba_drain()
        capi.synchronize()
        if not sg.status()[0]:
            raise SystemExit(f"bench: SuperGlue device path failed during warmup: {sg.error}")
        if dist:
            dist.barrier()
        sp.profile(True)  # (resets the stage accumulators)
        sg.profile(True)
        ba_ms.clear()
        ba_iters.clear()
        line_timers[:] = [capi.Timer() for _ in range(args.steps)]
        line_stats["detect_ms"].clear()
        line_stats["lines"].clear()
        line_t0 = args.warmup
        for k in host_wait:
            host_wait[k] = 0.0
        ba.kernel_times()  # reset
        ba.trace()  # reset (warmup calls)
        step_tr.clear()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + i)
        t_fed = time.perf_counter()
        ba_drain()
        t_drained = time.perf_counter()
        capi.synchronize()
        t_end = time.perf_counter()
        gc.enable()
        gc.unfreeze()
        elapsed = job_time(t_end - t0, dist)
        if trace_on:  # the timed region's host timeline, relative to its start (ms)
            rel = lambda t: round((t - t0) * 1e3, 4)  # noqa: E731
            trace_out.append({"precision": precision, "steps": args.steps, "warmup": args.warmup,
                              "elapsed_ms": rel(t_end), "fed_ms": rel(t_fed), "drained_ms": rel(t_drained),
                              "step": [{k: (v if k == "i" else rel(v)) for k, v in r.items()} for r in step_tr],
                              "ba": [{k: (rel(v) if k in ("submit", "stage0", "stage1", "run0", "upload", "opt1",
                                                          "opt2", "end") else v) for k, v in r.items()}
                                     for r in ba.trace()]})
        if ba_err:
            raise ba_err[0]
        # measurements of the timed region, read before the instrumented pass adds to them
        ba_ms_timed, ba_iters_timed = list(ba_ms), list(ba_iters)
        host_wait_timed = {k: round(v * 1e3 / args.steps, 4) for k, v in host_wait.items()}
        sp_ms, sp_calls = sp.stage_times()
        sg_ms, sg_calls = sg.stage_times()
        lines_ms = float(np.mean([tm.elapsed_ms() for tm in line_timers[:len(line_stats["detect_ms"])]])) \
            if line_stats["detect_ms"] else None
        lines_detect = float(np.mean(line_stats["detect_ms"])) if line_stats["detect_ms"] else None
        lines_per_step = float(np.mean(line_stats["lines"])) if line_stats["lines"] else None
        line_t0 = None
        # instrumented pass (untimed): the same steps with HIP events around the BA's two per-trial launches on
        # every call, for the BA rows of stages_roofline
        ba_kt, ba_timed_calls = None, 0
        if kt_steps > 0 and "ba" not in args.skip.split(","):
            ba.kernel_timing(1)
            ba.kernel_times()  # reset
            for i in range(kt_steps):
                step(args.warmup + args.steps + i)
            ba_drain()
            capi.synchronize()
            ba_kt = ba.kernel_times()
            ba.kernel_timing(0)
            ba_timed_calls = kt_steps * (world if shard else 1)
        if not native:
            ba_q.put(None)
            worker.join()
        if ba_err:
            raise ba_err[0]
        ok, mask = sg.status()  # Sinkhorn exchange health of every call in the timed region
        if not ok:
            raise SystemExit(f"bench: SuperGlue device path failed in the timed region (pairs 0x{mask:x}): {sg.error}")
        if dist:
            dist.barrier()

        if lm.status():
            raise SystemExit("bench: the stereo line association overflowed its point-line pairs")
        value = job_value(world, args.steps, elapsed)
        return {"value": value, "elapsed": elapsed, "sp": (sp_ms, sp_calls), "sg": (sg_ms, sg_calls),
                "stages": (sp, sg), "ba_ms": ba_ms_timed, "ba_iters": ba_iters_timed, "lines_ms": lines_ms,
                "lines_detect_ms": lines_detect, "lines_per_step": lines_per_step,
                "ba_kt": ba_kt, "ba_timed_calls": ba_timed_calls, "host_wait_ms": host_wait_timed}

    res = measure(args.precision)
    other = measure(precs[1]) if len(precs) > 1 else None  # the other precision, same run, for the record
    if trace_on:
        pathlib.Path(trace_path).write_text(json.dumps(trace_out))
    value, elapsed, ba_ms = res["value"], res["elapsed"], res["ba_ms"]
    sp_ms, sp_calls = res["sp"]
    sg_ms, sg_calls = res["sg"]
    sp, sg = res["stages"]
    if rank != 0:
        return
    stages = stage_roofline(sp, sg, sp_ms, sp_calls, sg_ms, sg_calls, args.precision, args.workload)
    if not shard and res["ba_kt"]:
        stages.update(ba_kernel_rows(problems[0], res["ba_kt"], res["ba_timed_calls"], args.workload))
    # the step-setting kernel: the largest device time per step over every timed kernel, the BA's
    # launches included (its launches per call x one call per step)
    dom_key = max((k for k in stages if stages[k]["single_kernel"]), key=lambda k: stages[k]["ms"])
    dom = {k: v for k, v in stages[dom_key].items() if k not in ("single_kernel",)}
    dom["ms_per_step"] = dom.pop("ms")
    traffic, traffic_src = pmc_traffic(dom["pmc_kernel"], args.workload)
    dom["traffic"] = round(traffic) if traffic else None
    dom["traffic_note"] = (f"HBM bytes per launch, rocprofv3 FETCH_SIZE(x2)+WRITE_SIZE, profiles/{traffic_src}"
                           if traffic else "no PMC summary for this kernel under profiles/")
    ba_wall = float(np.mean(ba_ms)) if ba_ms else None
    ba_it = float(np.mean(res["ba_iters"])) if res["ba_iters"] else None
    ba_bytes = float(np.mean([ba_bytes_per_iteration(p) for p in problems]))
    out = {
        "metric": {"c3": "stereo frames/sec SuperPoint+SuperGlue+localBA @752x480 (all-keyframe: 2xSP, 2xSG, 1 BA per frame)",
                   "c4": "stereo frames/sec SuperPoint+SuperGlue+localBA @640x512 (C4, all-keyframe: 2xSP, 2xSG, 1 BA per frame)",
                   "c5": "stereo frames/sec SuperPoint+SuperGlue+localBA @1920x1080 (C5, all-keyframe: 2xSP, 2xSG, 1 BA per frame)"
                   }[args.workload],
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"fp16": "fp16 MFMA with fp32 accumulation for SuperPoint/SuperGlue (the reference's TensorRT kFP16 "
                          "engines), fp32 Sinkhorn/decode, fp64 BA",
                  "fp16x3": "SuperPoint split fp16 (hi + lo operands, three fp16 MFMA products, fp32 accumulation: "
                            "fp32-grade results), SuperGlue fp16 MFMA with fp32 accumulation (the reference's TensorRT "
                            "kFP16), fp32 Sinkhorn/decode, fp64 BA",
                  "fp32": "fp32 (SuperPoint/SuperGlue MFMA), fp64 (BA)"}[args.precision],
        "data": f"synthetic (seeded textured stereo {W}x{H}, seeded weights, synthetic local-BA problems)",
        "config": {"workload": wl["desc"], "global_batch": world,
                   "parallelism": (f"replicas x{world} (one sequence per GPU)" if not shard else
                                   f"replicas x{world} front end; every step's {world} local BAs landmark-sharded "
                                   f"over {world} ranks (RCCL all-reduce per LM trial)"),
                   "python_gc": "cyclic GC frozen and disabled for the warmup and timed steps (reference counting "
                                "still frees; the feature loop is a Python driver, the reference's is C++)"},
        "roofline": {"kernel": dom_key, **dom},
        "stages_roofline": stages,
        "stages_ms_per_step": {**{f"sp:{n}": round(v / max(1, sp_calls), 4) for n, v in zip(sp.STAGES, sp_ms)},
                               **{f"sg:{n}": round(v / max(1, sg_calls), 4) for n, v in zip(sg.STAGES, sg_ms)},
                               "lines:detect": round(res["lines_detect_ms"], 4) if res["lines_detect_ms"] else None,
                               "lines:stereo": round(res["lines_ms"], 4) if res["lines_ms"] else None,
                               "ba:wall": round(ba_wall, 4) if ba_wall else None},
        # feature thread per step: blocked on the line threads / the BA queue, and its own SP / SG / association calls
        "host_ms_per_step": res["host_wait_ms"],
        "lines": {"lines_per_step": res["lines_per_step"], "keypoints_per_image": K,
                  "note": "lines:detect = per keyframe, the longer of the two images' LineDetector::LineExtractor jobs "
                          "on the RCF-like edge maps (restated FLD: GPU Canny classes + host chaining / fitting / "
                          "merges), each on its detector handle's native worker thread beside SP/SG "
                          "(rspl_lines_extract_async), joined before the association; lines:stereo = the stereo line "
                          "association on the GPU (AssignPointsToLines x2, disparity filter, MatchLines; "
                          "frame.cc:150-203), post stream, HIP-event time per step"},
        "ba": {"ms_per_call": round(ba_wall, 4) if ba_wall else None,
               "lm_iterations_per_call": ba_it,
               "us_per_lm_iteration": round(1e3 * ba_wall / ba_it, 2) if ba_wall and ba_it else None,
               "algorithmic_bytes_per_iteration": round(ba_bytes),
               "achieved_GBps": round(ba_bytes / (ba_wall / ba_it) / 1e6, 3) if ba_wall and ba_it else None,
               "frac_hbm": round(ba_bytes / (ba_wall / ba_it) / 1e6 / HBM_PEAK_GBS, 6) if ba_wall and ba_it else None,
               "note": "SURVEY 8(d) bytes per LM iteration; the BA is launch/latency-bound, wall time under the "
                       "pipeline's contention, host-array hand-over included"},
    }
    if other is not None:
        oname = other_prec[args.precision]
        out[f"{oname}_run"] = {"value": round(other["value"], 3),
                               "ms_per_step": round(1e3 * other["elapsed"] / args.steps, 3),
                               "note": "same workload and run, SP/SG at " + oname +
                                       {"fp32": " (the bit-parity path)",
                                        "fp16x3": " (SuperPoint split fp16: the fp32 keypoint sets; SuperGlue fp16)",
                                        "fp16": ""}[oname]}
    if world == 1 and not args.no_cpu_baseline:
        nproc = os.cpu_count() or 1
        threads = min(16, nproc)  # the GPU box's CPU share is 16 cores per GPU
        frames = args.cpu_frames or (12 if args.workload == "c3" else 1)
        cb = cpu_baseline(sp_w, sg_w, frames, threads, wl)
        cb1 = cpu_baseline(sp_w, sg_w, max(1, frames // 6), 1, wl)
        cb["nproc"] = nproc
        cb["one_core"] = {"value": cb1["value"], "cores": 1, "sample": cb1["sample"]}
        out["cpu_baseline"] = cb
        if args.workload == "c3":
            out["ate"] = ate_report(ba)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
