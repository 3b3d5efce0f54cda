"""Per-pass view of a batch-1 kernel trace (tools/gpu_b1_prof.sh): the timed
forward passes are the last STEPS repetitions of the same dispatch sequence;
report launches per pass, kernel-busy time per pass, the gaps between
dispatches, and the top kernels per pass.
usage: python tools/b1_trace_summ.py TRACE.csv [STEPS] [--seq]
--seq: also list one pass in dispatch order (grid, workgroup, mean duration of
that position over the timed passes)"""
import csv
import collections
import sys


def main():
    rows = list(csv.DictReader(open([a for a in sys.argv[1:] if not a.startswith("--")][0])))
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[1]) if len(args) > 1 else 20
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # the pass length: the smallest period P under which the last quarter of
    # the trace repeats (bench.py ends with the timed passes, the same passes
    # on one context, and one fully profiled pass; the setup's launches --
    # keygen, the transforms' diagonal encodes -- come first); the timed
    # passes are the STEPS periods before the final (profiled) one
    n = len(names)
    per = None
    lo = n - n // 4
    for P in range(20, n // 6):
        hi = n - P
        if hi > lo and sum(names[i] == names[i + P] for i in range(lo, hi)) >= 0.995 * (hi - lo):
            per = P
            break
    if per is None:
        raise SystemExit("no period found")
    end = n - per
    last = rows[end - per * steps:end]
    t0, t1 = int(last[0]["Start_Timestamp"]), int(last[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last)
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(last, last[1:])]
    print(f"launches per pass {per}; wall per pass {(t1 - t0) / steps / 1e3:.1f} us; "
          f"kernel busy per pass {busy / steps / 1e3:.1f} us; mean gap {sum(gaps) / len(gaps) / 1e3:.2f} us")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in last:
        short = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[short][0] += 1
        agg[short][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{n / steps:6.1f} x {ns / n / 1e3:6.2f} us = {ns / steps / 1e3:7.1f} us/pass  {k}")
    if "--seq" in sys.argv:
        print("\npos  grid  wg  mean_us  kernel")
        for i in range(per):
            rs = [last[i + k * per] for k in range(steps)]
            us = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / steps / 1e3
            r = rs[0]
            short = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            w = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
            print(f"{i:3d} {g // max(w, 1):6d} {w:4d} {us:8.2f}  {short}")


if __name__ == "__main__":
    main()
