"""Kernel timeline from a rocprofv3 --kernel-trace CSV: every launch of the
last N rounds (a round = from one solver launch to the next) with its start,
end and duration in microseconds relative to the round's solver start, and
its queue, so overlaps between the main stream and the side streams show.

    python3 tools/timeline.py gpurun_out/rocprof_TAG [rounds]
"""
import csv
import glob
import os
import sys


def short(name):
    for key, tag in (("solver_gram", "solver"), ("gram_seq", "gram_seq"), ("gram_list", "gram_list"), ("gram_kernel", "gram"), ("xw_produce", "xw"),
                     ("eval_stream", "eval"), ("eval_final", "eval_fin"), ("plan_kernel", "plan"),
                     ("fold", "fold"), ("sampler", "sampler"), ("copyBuffer", "copy"), ("fillBuffer", "fill")):
        if key in name:
            return tag
    return name[:24]


def main():
    d = sys.argv[1]
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    path = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), q))
    ev.sort()
    starts = [s for s, _, k, _ in ev if k == "solver"]
    if len(starts) < nr + 1:
        print("too few solver launches", len(starts))
        return
    for i in range(len(starts) - nr - 1, len(starts) - 1):
        t0, t1 = starts[i], starts[i + 1]
        print(f"-- round from solver start {i}: {(t1 - t0) / 1e3:.1f} us to the next solver start")
        for s, e, k, q in ev:
            if e < t0 or s >= t1:
                continue
            print(f"   {k:10s} q={q:>3s} start {(s - t0) / 1e3:9.1f}  end {(e - t0) / 1e3:9.1f}  dur {(e - s) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
