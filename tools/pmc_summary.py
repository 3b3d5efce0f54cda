"""Summarise one rocprofv3 profiling round (tools/gpu_prof.sh) into profiles/.

Reads gpurun_out/prof_<tag>/ (kernel-trace stats + the FETCH_SIZE, WRITE_SIZE
and SQ counter passes) and writes
  profiles/<tag>_kernel_stats.csv   the rocprofv3 --stats summary, verbatim
  profiles/<tag>_pmc_summary.json   per-kernel counter totals and the NTT HBM
                                    traffic per algorithmic byte
  profiles/ntt_traffic.json         HBM bytes per NTT launch for bench.py

HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled.  Algorithmic bytes of an NTT call, two
models (the same two bench.py reports): strict = 16 N per
limb-transform; fused = 16 N + 8 N per epilogue operand or addend read (the
subtract-and-scale operand, the word a rotate-and-add store adds to; the
automorphism's scatter index is a batch-shared table, excluded like the
twiddles).  Both hold for the one-pass kernels and the two-pass pairs
(ntt2.hip) alike; the traffic ratio is taken against the fused bytes.  The one-pass
kernels are persistent (one workgroup per CU walks the jobs), so the
limb-transform count of a dispatch comes from the library's call log
(ORION_NTT_LOG, one file per pass: gpurun_out/prof_<tag>/ntt_log_<pass>.txt),
paired with the pass's NTT dispatches in issue order.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def window_positions(d):
    """[i0, i1): dispatch positions (issue order) of the timed inference in the
    kernel trace: the kernels between the last two idle gaps of > 0.4 s that
    tools/resnet_bench.py leaves around it under PROF_MARK=1."""
    tr = sorted(rows(os.path.join(d, "kt_kernel_trace.csv")), key=lambda r: int(r["Dispatch_Id"]))
    gaps = [i for i in range(1, len(tr))
            if int(tr[i]["Start_Timestamp"]) - int(tr[i - 1]["End_Timestamp"]) > 400_000_000]
    if len(gaps) < 2:
        raise RuntimeError("no PROF_MARK gaps in the kernel trace")
    return gaps[-2], gaps[-1]


def in_window(rs, key, pos):
    """Rows whose dispatch (in issue order) falls in positions [pos[0], pos[1])."""
    ids = sorted({int(r[key]) for r in rs})
    keep = set(ids[pos[0]:pos[1]])
    return [r for r in rs if int(r[key]) in keep]


def window_stats(d, path, pos):
    """rocprofv3 --stats columns for the kernels of the timed inference only."""
    tr = in_window(rows(os.path.join(d, "kt_kernel_trace.csv")), "Dispatch_Id", pos)
    agg = collections.defaultdict(list)
    for r in tr:
        agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values())
    with open(path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v)])


def main(tag, workload="lola_n15", batch=64, logn=15, resnet=False, out=None):
    """resnet: the ResNet-20 N=2^16 passes of tools/gpu_resnet_prof.sh (no NTT
    call log, no shared roofline files); out: output directory (default
    profiles/; on the GPU box a directory under gpurun_out/, since only that
    is copied back)."""
    d = os.path.join(ROOT, "gpurun_out", f"prof_rn16_{tag}" if resnet else f"prof_{tag}")
    out = out or os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    if resnet:
        workload, batch, logn, tag = "resnet20_n16", 1, 16, f"{tag}_rn16"
        pos = window_positions(d)
        window_stats(d, os.path.join(out, f"{tag}_kernel_stats.csv"), pos)
    else:
        shutil.copy(os.path.join(d, "kt_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    N = 1 << logn
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    ntt_alg = ntt_fetch = ntt_write = 0.0
    solo_alg = solo_fetch = solo_write = 0.0
    def ntt_log(name):
        """The pass's NTT calls in order (bench.py run with ORION_NTT_LOG):
        (dispatches, jobs, subtract-and-scale epilogue); marker lines skipped."""
        p = os.path.join(d, f"ntt_log_{name}.txt")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return [tuple(int(v) for v in ln.split()[:3]) for ln in f if ln.strip() and not ln.startswith("#")]

    def log_window(name, tag):
        """[c0, c1): the calls between the log's last "# <tag> begin" and
        "# <tag> end" markers (bench.py: "timed" = the timed steps, "single" =
        the timed steps of the whole batch on one pipeline, "solo" = one fully
        profiled step of it), or None."""
        p = os.path.join(d, f"ntt_log_{name}.txt")
        if not os.path.exists(p):
            return None
        i, c0, win = 0, None, None
        with open(p) as f:
            for ln in f:
                if ln.startswith(f"# {tag} begin"):
                    c0 = i
                elif ln.startswith(f"# {tag} end") and c0 is not None:
                    win = (c0, i)
                elif ln.strip() and not ln.startswith("#"):
                    i += 1
        return win

    # the log's epilogue field (backend.hip log_ntt; 0/1 in logs before the
    # automorphism epilogues): extra fused-model bytes per coefficient over the
    # 16 of a plain transform -- the subtract-and-scale operand (8) and the word
    # the scatter adds to (8); the scatter index is not counted
    EPI_BYTES = {0: 0.0, 1: 8.0, 2: 8.0, 3: 16.0}
    EPI_NAME = {0: "store", 1: "sub", 2: "sub-aut", 3: "sub-aut-acc"}

    def ntt_log_full(name):
        """(dispatches, jobs, sub, inv, pro, intjobs[, family]) per call (older logs: 3 fields)."""
        p = os.path.join(d, f"ntt_log_{name}.txt")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return [tuple(int(v) for v in ln.split()) for ln in f if ln.strip() and not ln.startswith("#")]

    def priced(dispatches, log):
        """Pair the pass's NTT dispatches (in issue order) with its logged calls:
        yields (call index, dispatch, algorithmic bytes of the call or None for
        the 2nd dispatch of a two-pass pair, jobs of the call)."""
        i = 0
        for call, (nd, jobs, sub) in enumerate(log):
            for k in range(nd):
                if i >= len(dispatches):
                    raise RuntimeError("NTT log longer than the dispatch list")
                alg = jobs * (16.0 + EPI_BYTES.get(sub, 8.0)) * N if k == 0 else None
                yield call, dispatches[i], alg, jobs
                i += 1
        if i != len(dispatches):
            raise RuntimeError(f"{len(dispatches)} NTT dispatches vs {i} logged")

    for name in ("pmc_fetch", "pmc_write", "pmc_sq"):
        p = os.path.join(d, f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rs = rows(p)
        if resnet:
            rs = in_window(rs, "Dispatch_Id", pos)
        for r in rs:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            v = float(r["Counter_Value"])
            per[k][r["Counter_Name"]] += v
            per[k]["_dispatches_" + name] += 1
        if name == "pmc_sq":
            continue
        # HBM bytes of the batched NTT calls (>= 64 limb-transforms) per
        # algorithmic byte: each call's counters (both dispatches of a two-pass
        # pair) against 16 N per limb-transform (24 N with the epilogue)
        disp = {}
        for r in rs:
            disp.setdefault(int(r["Dispatch_Id"]), []).append(r)
        order = [disp[i] for i in sorted(disp)]
        log = ntt_log(name)
        if log is None:
            continue
        cnt = "FETCH_SIZE" if name == "pmc_fetch" else "WRITE_SIZE"
        # the single-pipeline window the bench's roofline is taken on: "single"
        # (round 6: the K timed steps on one context), else "solo" (one profiled step)
        sw = log_window(name, "single") or log_window(name, "solo")
        for call, drs, alg, jobs in priced(order, log):
            if jobs < 64:
                continue
            v = sum(float(r["Counter_Value"]) for r in drs if r["Counter_Name"] == cnt)
            solo = sw is not None and sw[0] <= call < sw[1]
            if cnt == "FETCH_SIZE":
                ntt_fetch += 2 * v * 1024  # gfx950 counts half the bytes of wide reads
                ntt_alg += alg or 0.0
                if solo:
                    solo_fetch += 2 * v * 1024
                    solo_alg += alg or 0.0
            else:
                ntt_write += v * 1024
                if solo:
                    solo_write += v * 1024
    ratio = (ntt_fetch + ntt_write) / ntt_alg if ntt_alg else None
    ratio_solo = (solo_fetch + solo_write) / solo_alg if solo_alg else None
    # the batched NTT calls of the kernel trace, counted the way bench.py's HIP
    # events count them: one call = one one-pass dispatch or one two-pass pair,
    # duration = the dispatches' summed time, priced with the logged
    # limb-transform counts; setup calls (keygen, < 64 jobs) are excluded
    kt = os.path.join(d, "kt_kernel_trace.csv")
    # issue order (Dispatch_Id): with pipeline threads the kernels of two streams
    # start out of call order, but they are dispatched in it
    tr = sorted(rows(kt), key=lambda r: int(r["Dispatch_Id"])) if os.path.exists(kt) else []
    tr = [r for r in tr if "ntt" in r["Kernel_Name"]]
    n_l = 0
    n_us = n_b = n_s = 0.0
    klog = ntt_log("kt")
    win = log_window("kt", "timed")
    swin = log_window("kt", "single") or log_window("kt", "solo")
    rwin = "single" if log_window("kt", "single") else "solo"
    w_iv, w_b, w_s, w_l = [], 0.0, 0.0, 0
    s_us, s_b, s_s, s_l = 0.0, 0.0, 0.0, 0
    if klog is not None:
        for call, r, alg, jobs in priced(tr, klog):
            if win and win[0] <= call < win[1]:  # bench.py's timed steps: every NTT call counts
                w_iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
                if alg is not None:
                    w_l += 1
                    w_b += alg
                    w_s += 16.0 * N * jobs
            if swin and swin[0] <= call < swin[1]:  # the single-pipeline step the bench's roofline is taken on
                s_us += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                if alg is not None:
                    s_l += 1
                    s_b += alg
                    s_s += 16.0 * N * jobs
            if jobs < 64:
                continue
            n_us += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if alg is not None:
                n_l += 1
                n_b += alg
                n_s += 16.0 * N * jobs
    # the timed window: the wall-clock union of its NTT dispatch intervals (the
    # bench line's definition with pipeline threads) and their summed durations
    timed = None
    if w_iv:
        w_iv.sort()
        union = 0
        b, e = w_iv[0]
        for x0, x1 in w_iv[1:]:
            if x0 > e:
                union += e - b
                b, e = x0, x1
            else:
                e = max(e, x1)
        union += e - b
        summed = sum(x1 - x0 for x0, x1 in w_iv)
        timed = {"calls": w_l, "union_us": union / 1e3, "summed_us": summed / 1e3,
                 "strict_bytes": w_s, "fused_bytes": w_b,
                 "frac_strict_union": w_s / (union * 1e-9) / 1e9 / 8000.0 if union else None,
                 "frac_fused_union": w_b / (union * 1e-9) / 1e9 / 8000.0 if union else None,
                 "frac_strict_summed": w_s / (summed * 1e-9) / 1e9 / 8000.0 if summed else None}
    # NTT time by launch class (kt pass): direction, kernel (one-pass / two-pass
    # pair), epilogue, prologue, integer-path share, jobs in multiples of CUs
    # (all calls of >= 64 jobs; and the calls of the solo / timed windows alone)
    classes, classes_solo, classes_timed = {}, {}, {}
    full = ntt_log_full("kt")
    if klog is not None and full is not None and len(full[0]) >= 6:
        for call, r, alg, jobs in priced(tr, klog):
            f = full[call]
            fam = {1: "1pass", 2: "2pass", 3: "2pass-s", 4: "rows-only"}.get(f[6]) if len(f) >= 7 else None
            fam = fam or ("1pass" if f[0] == 1 else "2pass")
            key = (f"{'inv' if f[3] else 'fwd'} {fam} "
                   f"{EPI_NAME.get(f[2], 'sub')} pro{f[4]} int{round(f[5] / f[1], 2)} jobs{f[1]}")
            dst = [classes] if jobs >= 64 else []
            if swin and swin[0] <= call < swin[1]:
                dst.append(classes_solo)
            if win and win[0] <= call < win[1]:
                dst.append(classes_timed)
            for cl in dst:
                c = cl.setdefault(key, {"calls": 0, "us": 0.0, "bytes": 0.0, "strict_bytes": 0.0})
                c["us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                if alg is not None:
                    c["calls"] += 1
                    c["bytes"] += alg
                    c["strict_bytes"] += 16.0 * N * jobs
        for cl in (classes, classes_solo, classes_timed):
            for c in cl.values():
                c["GBps"] = round(c["bytes"] / (c["us"] * 1e-6) / 1e9, 1) if c["us"] else None
                c["GBps_strict"] = round(c["strict_bytes"] / (c["us"] * 1e-6) / 1e9, 1) if c["us"] else None
                c["us_per_call"] = round(c["us"] / max(c["calls"], 1), 1)
                c["us"] = round(c["us"], 1)
    trace = {"launches": n_l, "avg_launch_us": n_us / n_l if n_l else None,
             "algorithmic_bytes_per_launch": n_b / n_l if n_l else None,
             "strict_bytes_per_launch": n_s / n_l if n_l else None,
             "achieved_GBps": n_b / (n_us * 1e-6) / 1e9 if n_us else None,
             "achieved_GBps_strict": n_s / (n_us * 1e-6) / 1e9 if n_us else None,
             "frac_fused": n_b / (n_us * 1e-6) / 1e9 / 8000.0 if n_us else None,
             "frac_strict": n_s / (n_us * 1e-6) / 1e9 / 8000.0 if n_us else None,
             "timed_window": timed,
             "solo_window": {"window": rwin, "calls": s_l, "avg_launch_us": s_us / s_l if s_l else None,
                             "strict_bytes_per_launch": s_s / s_l if s_l else None,
                             "frac_strict": s_s / (s_us * 1e-6) / 1e9 / 8000.0 if s_us else None,
                             "frac_fused": s_b / (s_us * 1e-6) / 1e9 / 8000.0 if s_us else None}
             if s_l else None}
    # VALU roofline of the VALU-bound kernels: the fraction of SIMD cycles in
    # which a VALU instruction was executing, sum over waves of
    # SQ_ACTIVE_INST_VALU (quad-cycles, so x4) / (elapsed cycles x 1024 SIMDs);
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md), so the
    # elapsed cycles of the dispatches are GRBM_GUI_ACTIVE / 8.  Also the
    # achieved VALU wave-instruction rate against 1 per 2 cycles per SIMD (a
    # single-pass 32-bit op on SIMD32; 64-bit ops and u64 multiplies issue at
    # 1 per 4.5-5.3 cycles, tools/ubench/valu_rates.hip)
    valu = {}
    for k, v in per.items():
        g = v.get("GRBM_GUI_ACTIVE")
        if not g or "SQ_ACTIVE_INST_VALU" not in v:
            continue
        cyc = g / 8.0
        valu[k] = {"valu_busy": v["SQ_ACTIVE_INST_VALU"] * 4.0 / (cyc * 1024),
                   "valu_insts_per_simd_cycle": v["SQ_INSTS_VALU"] / (cyc * 1024),
                   "frac_of_single_pass_peak": v["SQ_INSTS_VALU"] / (cyc * 1024) * 2.0,
                   "wait_inst_any_per_wave_cycle": v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"]
                   if v.get("SQ_WAVE_CYCLES") else None,
                   "salu_per_valu_inst": v["SQ_INSTS_SALU"] / v["SQ_INSTS_VALU"]
                   if v.get("SQ_INSTS_SALU") and v.get("SQ_INSTS_VALU") else None}
    if valu and not resnet:
        with open(os.path.join(out, "valu_roofline.json"), "w") as f:
            json.dump({"tag": tag, "workload": workload, "batch": batch,
                       "definition": "valu_busy = sum SQ_ACTIVE_INST_VALU*4 / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
                       "kernels": valu}, f, indent=1)
    summary = {"tag": tag, "ntt_hbm_bytes_per_algorithmic_byte": ratio,
               "ntt_hbm_bytes_per_algorithmic_byte_solo": ratio_solo, "ntt_trace_batched": trace,
               "ntt_classes": dict(sorted(classes.items(), key=lambda kv: -kv[1]["us"])),
               "ntt_classes_solo": dict(sorted(classes_solo.items(), key=lambda kv: -kv[1]["us"])),
               "ntt_classes_timed": dict(sorted(classes_timed.items(), key=lambda kv: -kv[1]["us"])), "valu": valu,
               "ntt_fetch_bytes_per_algorithmic_byte": ntt_fetch / ntt_alg if ntt_alg else None,
               "kernels": {k: dict(v) for k, v in per.items()}}
    with open(os.path.join(out, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if ratio and not resnet:
        with open(os.path.join(out, "ntt_traffic.json"), "w") as f:
            json.dump({"tag": tag, "workload": workload, "batch": batch,
                       "hbm_bytes_per_algorithmic_byte": round(ratio, 4),
                       "hbm_bytes_per_algorithmic_byte_solo": round(ratio_solo, 4) if ratio_solo else None},
                      f, indent=1)
    print(json.dumps({"tag": tag, "ntt_hbm_bytes_per_algorithmic_byte": ratio, "ntt_trace_batched": trace}))


if __name__ == "__main__":
    a = sys.argv[1:]
    rn = "--resnet" in a
    a = [x for x in a if x != "--resnet"]
    main(a[0], resnet=rn, out=a[1] if len(a) > 1 else None)
