"""NTT kernel microbenchmark (GPU): per-launch time and algorithmic GB/s
(16 N bytes per limb-transform) for the float64 path (40-bit moduli), the
integer path (60-bit moduli) and a LoLA-like mix, at several job counts.
Usage: python tools/ntt_bench.py   (env: LOGN, JOBS, ORION_LIB, TAG, OOP=1 out-of-place forward;
ORION_NTT_ORDER selects the job order of the library under test)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.backend import HipLibrary  # noqa: E402


def main():
    logn = int(os.environ.get("LOGN", 15))
    N = 1 << logn
    path = os.environ.get("ORION_LIB")
    lib = (HipLibrary(path) if path else HipLibrary()).new_scheme(logn, [40] * 8 + [60] * 8, [60], 40)
    mods = lib.moduli()
    res = []
    kinds = [("f64(40-bit)", list(range(0, 8))), ("int(60-bit)", list(range(8, 16))),
             ("mix(5:3)", [8, 0, 1, 2, 3, 4, 9, 10])]
    only = os.environ.get("KINDS")
    if only:
        kinds = [k for k in kinds if k[0].split("(")[0] in only.split(",")]
    oop = os.environ.get("OOP") == "1"  # forward out of place (the half-limb kernel's launches)
    for kind, mset in kinds:
        for jobs in [int(j) for j in os.environ.get("JOBS", "256,1024,4096").split(",")]:
            nl = len(mset)
            B = jobs // nl
            rng = np.random.default_rng(0)
            host = np.stack([rng.integers(0, mods[m], (B, N), dtype=np.uint64) for m in mset])
            if oop:  # out of place: results into a second buffer right after the input
                host = np.concatenate([host, np.zeros_like(host)])
            dev = torch.from_numpy(host.view(np.int64)).cuda()
            ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
            mc = (ctypes.c_int * nl)(*mset)
            for inv in (0, 1):
                for _ in range(3):
                    lib.lib.OrionHipNTT(ptr, nl, B, mc, inv | (2 if oop and not inv else 0))
                lib.OrionHipSynchronize()
                s = torch.cuda.Stream(device=0)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                lib.OrionHipSetStream(s.cuda_stream)
                reps = 10
                with torch.cuda.stream(s):
                    e0.record(s)
                    for _ in range(reps):
                        lib.lib.OrionHipNTT(ptr, nl, B, mc, inv | (2 if oop and not inv else 0))
                    e1.record(s)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                gbs = 16 * N * jobs / (ms * 1e-3) / 1e9
                line = (f"{kind:12s} {'inv' if inv else 'fwd'} jobs={jobs:5d}  {ms*1e3:8.1f} us/launch  "
                        f"{gbs:7.1f} GB/s  {ms*1e3/(jobs/256):6.1f} us per 256 limbs")
                print(line, flush=True)
                res.append(line)
            del dev
    tag = os.environ.get("TAG", "")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"ntt_bench_{logn}{tag}.txt"), "w") as f:
        f.write("\n".join(res) + "\n")


if __name__ == "__main__":
    main()
