#!/usr/bin/env python3
"""Headline benchmark: stereo frames/sec through SuperPoint -> SuperGlue -> local BA @ 752x480.

Workload (BASELINE.json configs[2], "C3", all-keyframe worst case of SURVEY.md §8d): every
step is one stereo keyframe of a synthetic EuRoC-shaped stream:
  * SuperPoint on the rectified stereo pair (batch 2, 480x752, top-400),
  * SuperGlue/PointMatching on 2 pairs: left(t) vs left(t-1) keyframe, left(t) vs right(t),
  * one local BA (LocalmapOptimization) of a C3-sized problem: 10 keyframes (1 fixed),
    ~4k points / ~10^4 point observations, 100 lines (synthetic, with ground truth).
Inputs (images) are resident in HBM before timing.  BA is host-driven and runs on its own
(highest-priority) stream, overlapping the frame's SP/SG exactly as the reference's tracking
thread overlaps its feature thread (src/map_builder.cc:48-49); SP of frame t+1 runs on its own
stream beside SG of frame t (event-ordered).  The timed region ends with a device
synchronisation, so every frame's SP, SG and BA work is inside it.  The BA problem is handed over as host
arrays (the reference's std::map containers), so its H2D upload is inside the step.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU, each
rank runs its own stereo sequence (replicas, weak scaling, no data-path collective); the
gloo process group only provides the barrier and the max-over-ranks timing, so a single
HIP runtime (librspl's system ROCm) drives each GPU.
"""
import argparse
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

H, W, K = 480, 752, 400
FP32_MFMA_PEAK = 157.3  # TFLOP/s, MI355X_MICROARCH.md (v_mfma_f32_32x32x2_f32, dense)
FP16_MFMA_PEAK = 2516.8  # TFLOP/s dense (~2.5 PF, = 16 x the f32 MFMA rate), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0  # HBM3E, MI355X_MICROARCH.md
CONV1_GFLOP_PER_IMAGE = 2 * H * W * 64 * 9 / 1e9 + 2 * H * W * 64 * 576 / 1e9  # conv1a + conv1b


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def cpu_baseline(sp_w, sg_w, frames, threads):
    """The oracle's C restatement (oracle/*.c) of the same per-keyframe work on host cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # checker/baseline only
    import post
    oracle.set_threads(threads)
    syn = pkg.synthetic
    probs = [syn.ba_problem(n_poses=10, n_points=4000, n_lines=100, seed=100 + i)[0] for i in range(frames)]
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


def pmc_traffic(kernel_substr):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from two rocprofv3
    --pmc passes, FETCH_SIZE x2 gfx950 correction), or None."""
    for f in sorted((ROOT / "profiles").glob("*_pmc_traffic*.json"), reverse=True):  # newest first
        for name, v in json.loads(f.read_text()).items():
            if kernel_substr in name:
                return v["traffic_bytes"], f.name
    return None, None


def stage_roofline(sp, sg, sp_ms, sp_calls, sg_ms, sg_calls, precision):
    """Achieved rate vs the bounding peak for the other big stages (HIP-event stage times, per
    step: 2 SuperPoint images, 2 SuperGlue pairs of N = M = 400).  Algorithmic work as SURVEY.md
    8(d): GNN 2*(655,360 N + 512 N M) per image per layer; Sinkhorn streamed model
    2*iters*4*(N+1)(M+1) bytes per pair; NMS 2*4*H*W bytes per image."""
    t = {**{f"sp:{n}": v / max(1, sp_calls) for n, v in zip(sp.STAGES, sp_ms)},
         **{f"sg:{n}": v / max(1, sg_calls) for n, v in zip(sg.STAGES, sg_ms)}}
    N = M = K
    mfma_peak = FP16_MFMA_PEAK if precision == "fp16" else FP32_MFMA_PEAK
    gnn_gflop = 2 * 2 * 18 * 2 * (655360 * N + 512 * N * M) / 1e9
    sink_gb = 2 * 2 * 100 * 4 * (N + 1) * (M + 1) / 1e9
    nms_gb = 2 * 2 * 4 * H * W / 1e9
    out = {}
    for key, work, unit, peak, bound in (("sg:gnn x18", gnn_gflop, "TFLOP/s", mfma_peak, "mfma"),
                                         ("sg:sinkhorn", sink_gb, "GB/s", HBM_PEAK_GBS, "hbm (latency)"),
                                         ("sp:nms", nms_gb, "GB/s", HBM_PEAK_GBS, "hbm (latency)")):
        ms = t.get(key)
        if ms:
            ach = work / ms if unit == "TFLOP/s" else work / ms * 1e3
            out[key] = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                        "frac": round(ach / peak, 4), "ms": round(ms, 4)}
    return out


def ate_report(ba, ba_sets):
    """'ATE vs ref' at the BA level on the bench's own C3 problems: RMS distance between the
    keyframe positions the GPU BA returns and (a) those of the reference-algorithm restatement
    (oracle/ba.c, the g2o LocalmapOptimization restatement) on the same inputs, (b) the synthetic
    ground truth; (c) the ground-truth error of the perturbed initial estimate, for scale.  Optimised
    (non-fixed) poses only.  A trajectory-level ATE needs the reference's map/tracking control plane
    and datasets, out of scope here."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # checker only
    d_ref, d_gt, d_init = [], [], []
    for prob, gt in ba_sets:
        res, ref = ba.run(prob), oracle.ba_local(prob)
        free = prob.pose_fixed == 0
        d_ref.append(np.linalg.norm(res.pose_p[free] - ref.pose_p[free], axis=1))
        d_gt.append(np.linalg.norm(res.pose_p[free] - gt["pose_p"][free], axis=1))
        d_init.append(np.linalg.norm(prob.pose_p[free] - gt["pose_p"][free], axis=1))
    rms = lambda d: float(np.sqrt(np.mean(np.concatenate(d) ** 2)))
    return {"vs_reference_restatement_m": rms(d_ref), "vs_ground_truth_m": rms(d_gt),
            "initial_vs_ground_truth_m": rms(d_init), "problems": len(ba_sets),
            "note": "BA-level keyframe-position RMS on the bench's synthetic C3 problems (not a dataset trajectory)"}


def replica_seeds(rank):
    """Per-rank synthetic sequence (replicas: each GPU runs its own stereo stream)."""
    return {"images": [1000 * rank + i for i in range(4)], "ba": [1000 * rank + 50 + i for i in range(3)]}


def job_time(elapsed, dist=None):
    """Whole-job wall time = max over ranks of each rank's timed region (gloo all-reduce)."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def job_value(world, steps, elapsed):
    """frames/s over all ranks: every rank processed `steps` stereo keyframes."""
    return world * steps / elapsed


def main():
    capi.load()  # librspl's HIP runtime first: one runtime per process
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-frames", type=int, default=12, help="keyframes in the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", choices=["fp32", "fp16"], default="fp16",
                    help="SP/SG MFMA precision: fp16 = the reference's own TensorRT kFP16 engines "
                         "(src/super_point.cpp:98, src/super_glue.cpp:132; default), fp32 = the parity path")
    ap.add_argument("--reserve-cus", type=int, default=int(os.environ.get("RSPL_RESERVE_CUS", "0")),
                    help="CUs the SuperPoint/SuperGlue streams leave free for the BA chain (CU-masked streams)")
    ap.add_argument("--ba-own-cus", type=int, default=int(os.environ.get("RSPL_BA_OWN_CUS", "1")),
                    help="1: the BA runs only on the reserved CUs (disjoint from SP/SG)")
    ap.add_argument("--skip", default="", help="diagnostics only: comma list of stages to leave out (sp,sg,ba)")
    ap.add_argument("--single-precision", action="store_true",
                    help="skip the second (other-precision) measurement")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    capi.check(capi.load().rspl_set_device(local), "rspl_set_device")

    sp_w, sg_w = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    precs = [args.precision] + (["fp32" if args.precision == "fp16" else "fp16"]
                                if world == 1 and not args.single_precision else [])
    handles = {}
    for pr in precs:  # all handles and streams created once, up front: fixed HW-queue placement
        code = capi.RSPL_PREC_FP16 if pr == "fp16" else capi.RSPL_PREC_FP32
        sp_h = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=K, weights=sp_w, max_height=H, max_width=W,
                                                   max_batch=2, precision=code, device=local))
        assert sp_h.build(), sp_h.error
        sg_h = pkg.SuperGlue(pkg.SuperGlueConfig(image_width=W, image_height=H, weights=sg_w, max_keypoints=K,
                                                 max_batch=2, precision=code, device=local))
        assert sg_h.build(), sg_h.error
        handles[pr] = (sp_h, sg_h)
    ba = pkg.LocalBA(max_poses=16, max_points=6000, max_lines=200, max_edges=40000, device=local)
    if args.ba_own_cus and args.reserve_cus > 0:
        ba.use_reserved_cus(args.reserve_cus)
    syn = pkg.synthetic
    NP = 4
    pool = capi.DeviceBuffer(NP * 2 * H * W)
    seeds = replica_seeds(rank)
    for i in range(NP):
        L, R = syn.stereo_pair(H, W, seed=seeds["images"][i])
        pool.upload(np.stack([L, R]), offset=i * 2 * H * W)
    ba_sets = [syn.ba_problem(n_poses=10, n_points=4000, n_lines=100, seed=sd) for sd in seeds["ba"]]
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
    # under load (1.62 -> 1.90 ms of GPU work) is memory-latency contention, not CU slots -- so the
    # default is 0 (unmasked)
    rc = args.reserve_cus
    # stream priorities (RSPL_STREAM_PRIO="sp=normal,sg=high,post=high", the defaults): the BA's
    # own stream is always high
    prio = dict(sp="normal", sg="high", post="high")
    prio.update(kv.split("=") for kv in os.environ.get("RSPL_STREAM_PRIO", "").split(",") if "=" in kv)
    st_sp, st_sg = capi.Stream(reserve_cus=rc, priority=prio["sp"]), capi.Stream(reserve_cus=rc, priority=prio["sg"])
    st_post = capi.Stream(reserve_cus=rc, priority=prio["post"])  # SG's Sinkhorn + decode: overlaps the next GNN
    ev_sp = [capi.Event() for _ in range(3)]
    ev_sg = [capi.Event() for _ in range(3)]

    def measure(precision):
        """One full timed run of the pipeline at `precision`; returns its measurements."""
        sp, sg = handles[precision]
        for c in counts:
            c.zero()
        capi.synchronize()
        ba_ms = []
        ba_err = []
        ba_q = queue.Queue(maxsize=2)

        def tracking_thread():
            """BA worker: the reference runs LocalmapOptimization on the tracking thread while the
            feature thread keeps extracting/matching (src/map_builder.cc:48-49, src/map.cc:105-107)."""
            capi.check(capi.load().rspl_set_device(local), "rspl_set_device")  # HIP device is per thread
            while True:
                prob = ba_q.get()
                if prob is None:
                    ba_q.task_done()
                    return
                t = time.perf_counter()
                try:
                    ba.run(prob)
                except Exception as e:  # surfaced on the main thread
                    ba_err.append(e)
                ba_ms.append((time.perf_counter() - t) * 1e3)
                ba_q.task_done()

        worker = threading.Thread(target=tracking_thread, daemon=True)
        worker.start()

        def step(i):
            slot, pslot = i % 3, (i - 1) % 3
            cur, prev, ccur, cprev = feats[slot], feats[pslot], counts[slot], counts[pslot]
            skip = args.skip.split(",")
            if "sp" in skip or "sg" in skip:  # diagnostics: stages left out (not a benchmark line)
                if "sp" not in skip:
                    sp.infer_device(pool.offset((i % NP) * 2 * H * W), 2, H, W, W, H * W, cur.ptr, K, ccur.ptr,
                                    st_sp.handle)
                if "sg" not in skip:
                    sg.infer_device(2, f0.ptr, n0.ptr, f1.ptr, n1.ptr, K, True, outs[0].ptr, outs[1].ptr,
                                    outs[2].ptr, outs[3].ptr, st_sg.handle, post_stream=st_post.handle)
                if "ba" not in skip:
                    ba_q.put(problems[i % len(problems)])
                return
            if i >= 2:
                ev_sg[(i - 2) % 3].wait_on(st_sp.handle)
            sp.infer_device(pool.offset((i % NP) * 2 * H * W), 2, H, W, W, H * W, cur.ptr, K, ccur.ptr, st_sp.handle)
            ev_sp[slot].record(st_sp.handle)
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
            ev_sg[slot].record(st_post.handle)  # matches complete on the post stream
            # keyframe i's local BA goes to the tracking thread (own high-priority stream) through a
            # 2-deep buffer, as the reference's feature thread blocks only while
            # _tracking_data_buffer.size() >= 2 (src/map_builder.cc:176)
            ba_q.put(problems[i % len(problems)])

        for i in range(args.warmup):
            step(i)
        ba_q.join()
        capi.synchronize()
        if dist:
            dist.barrier()
        sp.profile(True)
        sg.profile(True)
        ba_ms.clear()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + i)
        ba_q.join()
        capi.synchronize()
        elapsed = job_time(time.perf_counter() - t0, dist)
        ba_q.put(None)
        worker.join()
        if ba_err:
            raise ba_err[0]
        if dist:
            dist.barrier()

        sp_ms, sp_calls = sp.stage_times()
        sg_ms, sg_calls = sg.stage_times()
        conv1_ms = sp_ms[0] / max(1, sp_calls)
        achieved = 2 * CONV1_GFLOP_PER_IMAGE / conv1_ms  # GFLOP / ms = TFLOP/s
        value = job_value(world, args.steps, elapsed)
        return {"value": value, "elapsed": elapsed, "sp": (sp_ms, sp_calls), "sg": (sg_ms, sg_calls), "stages": (sp, sg),
                "conv1_ms": conv1_ms, "achieved": achieved, "ba_ms": list(ba_ms)}

    res = measure(args.precision)
    other = measure(precs[1]) if len(precs) > 1 else None  # the other precision, same run, for the record
    value, elapsed, conv1_ms, achieved, ba_ms = (res["value"], res["elapsed"], res["conv1_ms"], res["achieved"],
                                                 res["ba_ms"])
    sp_ms, sp_calls = res["sp"]
    sg_ms, sg_calls = res["sg"]
    sp, sg = res["stages"]
    traffic, traffic_src = pmc_traffic("conv3x3_kernel<64, 16, true, true>" if args.precision == "fp32"
                                       else "conv3x3_h_kernel<64, 16, true, true, false>")
    if rank != 0:
        return
    peak = FP16_MFMA_PEAK if args.precision == "fp16" else FP32_MFMA_PEAK
    out = {
        "metric": "stereo frames/sec SuperPoint+SuperGlue+localBA @752x480 (all-keyframe: 2xSP, 2xSG, 1 BA per frame)",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp16 MFMA with fp32 accumulation for SuperPoint/SuperGlue (the reference's TensorRT kFP16 "
                  "engines), fp32 Sinkhorn/decode, fp64 BA") if args.precision == "fp16"
                 else "fp32 (SuperPoint/SuperGlue MFMA), fp64 (BA)",
        "data": "synthetic (seeded textured stereo 752x480, seeded weights, synthetic C3 local-BA problems)",
        "config": {"workload": "C3 EuRoC 752x480 stereo keyframe stream: SP batch 2 top-400, SG 2 pairs N=400, "
                               "local BA 10 poses / ~4k points / 100 lines",
                   "global_batch": world, "parallelism": f"replicas x{world} (one sequence per GPU)"},
        "roofline": {"kernel": ("conv3x3_h_kernel<64,16,true,true,false>" if args.precision == "fp16"
                                else "conv3x3_kernel<64,16,true,true>") + " (conv1a+conv1b+ReLU+pool, fused)",
                     "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4),
                     "traffic": round(traffic) if traffic else None,
                     "traffic_note": (f"HBM bytes per launch, rocprofv3 FETCH_SIZE(x2)+WRITE_SIZE, {traffic_src}; "
                                      "algorithmic minimum = pooled 64-ch output (46.2 MB fp32 / 23.1 MB fp16) "
                                      "+ 0.7 MB images")
                     if traffic else None,
                     "algorithmic": f"{2 * CONV1_GFLOP_PER_IMAGE:.3f} GFLOP per launch (2 images)",
                     "avg_launch_ms": round(conv1_ms, 4)},
        "stages_roofline": stage_roofline(sp, sg, sp_ms, sp_calls, sg_ms, sg_calls, args.precision),
        "stages_ms_per_step": {**{f"sp:{n}": round(v / max(1, sp_calls), 4) for n, v in zip(sp.STAGES, sp_ms)},
                               **{f"sg:{n}": round(v / max(1, sg_calls), 4) for n, v in zip(sg.STAGES, sg_ms)},
                               "ba:wall": round(float(np.mean(ba_ms)), 4) if ba_ms else None},
    }
    if other is not None:
        oname = "fp32" if args.precision == "fp16" else "fp16"
        out[f"{oname}_run"] = {"value": round(other["value"], 3),
                               "ms_per_step": round(1e3 * other["elapsed"] / args.steps, 3),
                               "note": "same workload and run, SP/SG at " + oname +
                                       (" (the bit-parity path)" if oname == "fp32" else "")}
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(sp_w, sg_w, args.cpu_frames, threads)
        out["ate"] = ate_report(ba, ba_sets)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
