"""Summarise one rocprofv3 profiling round (tools/gpu_prof.sh) into profiles/.

Reads gpurun_out/prof_<tag>/ (kernel-trace stats + the FETCH_SIZE, WRITE_SIZE
and SQ counter passes) and writes
  profiles/<tag>_kernel_stats.csv   the rocprofv3 --stats summary, verbatim
  profiles/<tag>_pmc_summary.json   per-kernel counter totals and the NTT HBM
                                    traffic per algorithmic byte
  profiles/ntt_traffic.json         HBM bytes per NTT launch for bench.py

HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled.  Algorithmic bytes of an NTT launch =
16 N per limb-transform (24 N with the subtract-and-scale epilogue), for the
one-pass kernels (one workgroup of N/32 threads per limb) and the two-pass
pairs (ntt2.hip) alike.
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


def main(tag, workload="lola_n15", batch=64, logn=15):
    d = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(d, "kt_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    N = 1 << logn
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    ntt_alg = ntt_fetch = ntt_write = 0.0
    for name in ("pmc_fetch", "pmc_write", "pmc_sq"):
        p = os.path.join(d, f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in rows(p):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            v = float(r["Counter_Value"])
            per[k][r["Counter_Name"]] += v
            per[k]["_dispatches_" + name] += 1
            # algorithmic bytes of this dispatch (batched launches only, >= 64
            # jobs): one-pass kernel = jobs * 16 N (24 N with the subtract-and-
            # scale epilogue); a two-pass call's 16 N per job is booked on its
            # cols kernel, the epilogue's extra 8 N on its rows kernel
            wgs = int(r["Grid_Size"]) // max(1, int(r.get("Workgroup_Size") or 1))
            tmpl = k.split("<")[1].split(">")[0].replace(" ", "") if "<" in k else ""
            alg = None
            if "ntt2_" in k:
                jobs = wgs // 16 if "_cols" in k else wgs // (1 << (logn - 12))
                if jobs >= 64:
                    alg = jobs * 16.0 * N if "_cols" in k else (
                        jobs * 8.0 * N if ("ntt2_fwd_rows" in k and tmpl.endswith(",1")) else 0.0)
            elif "ntt_" in k and wgs >= 64:
                alg = wgs * (24.0 if ("ntt_fwd_kernel" in k and tmpl.endswith(",1")) else 16.0) * N
            if alg is not None:
                if r["Counter_Name"] == "FETCH_SIZE":
                    ntt_fetch += 2 * v * 1024
                    ntt_alg += alg
                elif r["Counter_Name"] == "WRITE_SIZE":
                    ntt_write += v * 1024
    ratio = (ntt_fetch + ntt_write) / ntt_alg if ntt_alg else None
    # the batched NTT launches of the kernel trace, counted the way bench.py's
    # HIP events count them: one launch per transform call, i.e. one one-pass
    # kernel (jobs = workgroups) or one two-pass pair (ntt2.hip: cols kernel
    # jobs*16 workgroups + rows kernel jobs*BTILES, BTILES = 2^(logn-12)),
    # duration = the kernels' summed time; setup launches (keygen, < 64 jobs)
    # are excluded
    tr = sorted(rows(os.path.join(d, "kt_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    btiles = 1 << (logn - 12)
    n_l = 0
    n_us = n_b = 0.0
    for r in tr:
        k = r["Kernel_Name"]
        if "ntt" not in k:
            continue
        wgs = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tmpl = k.split("<")[1].split(">")[0].replace(" ", "") if "<" in k else ""
        if "ntt2_" in k:
            cols = "_cols" in k
            jobs = wgs // 16 if cols else wgs // btiles
            if jobs < 64:
                continue
            n_us += dur
            if cols:
                n_l += 1
                n_b += jobs * 16.0 * N
            elif "ntt2_fwd_rows" in k and tmpl.endswith(",1"):  # subtract-and-scale epilogue
                n_b += jobs * 8.0 * N
            continue
        if "ntt_" not in k or wgs < 64:
            continue
        n_l += 1
        n_us += dur
        sub = "ntt_fwd_kernel<" in k and tmpl.endswith(",1")
        n_b += wgs * (24.0 if sub else 16.0) * N
    trace = {"launches": n_l, "avg_launch_us": n_us / n_l if n_l else None,
             "algorithmic_bytes_per_launch": n_b / n_l if n_l else None,
             "achieved_GBps": n_b / (n_us * 1e-6) / 1e9 if n_us else None}
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
                   if v.get("SQ_WAVE_CYCLES") else None}
    if valu:
        with open(os.path.join(out, "valu_roofline.json"), "w") as f:
            json.dump({"tag": tag, "workload": workload, "batch": batch,
                       "definition": "valu_busy = sum SQ_ACTIVE_INST_VALU*4 / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
                       "kernels": valu}, f, indent=1)
    summary = {"tag": tag, "ntt_hbm_bytes_per_algorithmic_byte": ratio, "ntt_trace_batched": trace, "valu": valu,
               "ntt_fetch_bytes_per_algorithmic_byte": ntt_fetch / ntt_alg if ntt_alg else None,
               "kernels": {k: dict(v) for k, v in per.items()}}
    with open(os.path.join(out, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if ratio:
        with open(os.path.join(out, "ntt_traffic.json"), "w") as f:
            json.dump({"tag": tag, "workload": workload, "batch": batch,
                       "hbm_bytes_per_algorithmic_byte": round(ratio, 4)}, f, indent=1)
    print(json.dumps({"tag": tag, "ntt_hbm_bytes_per_algorithmic_byte": ratio, "ntt_trace_batched": trace}))


if __name__ == "__main__":
    main(sys.argv[1])
