"""Summarise bench.py's host timeline (RSPL_BENCH_TRACE): per step the feature loop's marks, per BA call the
tracking / staging threads' (rspl_ba_trace).  Prints a table per run and the call-by-call BA timeline."""
import json
import sys

import numpy as np


def summarize(path, calls=False):
    runs = json.load(open(path))
    for r in runs:
        st, ba = r["step"], r["ba"]
        dur = np.diff([s["t"] for s in st] + [r["fed_ms"]])
        put = np.array([s.get("ba_put1", 0) - s.get("ba_put0", 0) for s in st])
        print(f"{path} [{r['precision']}] steps {r['steps']} elapsed {r['elapsed_ms']:.2f} ms "
              f"({r['elapsed_ms'] / r['steps']:.3f}/step), fed {r['fed_ms']:.2f}, drained {r['drained_ms']:.2f}")
        print(f"  step ms: mean {dur.mean():.3f} p50 {np.median(dur):.3f} max {dur.max():.3f}; "
              f"blocked on the BA queue: mean {put.mean():.3f} max {put.max():.3f}")
        if not ba:
            continue
        f = {k: np.array([c[k] for c in ba]) for k in ba[0]}
        run = f["end"] - f["run0"]
        gap = f["run0"][1:] - f["end"][:-1]
        print(f"  BA calls {len(ba)}: run ms mean {run.mean():.3f} p50 {np.median(run):.3f} max {run.max():.3f}; "
              f"idle gap before a call mean {gap.mean():.3f}; stage {np.mean(f['stage1'] - f['stage0']):.3f}; "
              f"upload {np.mean(f['upload'] - f['run0']):.3f} opt1 {np.mean(f['opt1'] - f['upload']):.3f} "
              f"opt2 {np.mean(f['opt2'] - f['opt1']):.3f} final {np.mean(f['end'] - f['opt2']):.3f}; "
              f"grew {int((f['grew'] != 0).sum())}")
        if calls:
            for i, c in enumerate(ba):
                print(f"    call {i}: submit {c['submit']:.3f} stage {c['stage0']:.3f}-{c['stage1']:.3f} run {c['run0']:.3f} "
                      f"up {c['upload'] - c['run0']:.3f} o1 {c['opt1'] - c['upload']:.3f} o2 {c['opt2'] - c['opt1']:.3f} "
                      f"fin {c['end'] - c['opt2']:.3f} = {c['end'] - c['run0']:.3f} slot {int(c['slot'])} grew {int(c['grew'])} "
                      f"it {int(c['iters'])}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        if p != "--calls":
            summarize(p, "--calls" in sys.argv)
