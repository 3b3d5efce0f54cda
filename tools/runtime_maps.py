"""Module map for the r03p SIGSEGV relocation: load
liborion_hip.so BEFORE torch, as tools/resnet_bench.py did at r03p (its
marker imported torch only after the library had initialised HIP), create a
scheme (HIP / HSA initialised by the library), dump /proc/self/maps, then
import torch and dump again.  No torch kernel is launched (the crash was the
first torch kernel launch), so this does not repeat the crashing step.
Run under `rocprofv3 --kernel-trace --` so the preloaded profiler libraries
sit where they sat in the crash run.

Usage: rocprofv3 --kernel-trace -d gpurun_out/maps -- python tools/runtime_maps.py OUTPREFIX
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dump(path):
    with open("/proc/self/maps") as f, open(path, "w") as o:
        o.write(f.read())


def main():
    prefix = sys.argv[1]
    lib = ctypes.CDLL(os.path.join(HERE, "orion_amd", "liborion_hip.so"))  # the r03p load order
    lib.OrionHipSetDevice.argtypes = [ctypes.c_int]
    if lib.OrionHipSetDevice(0) != 0:
        raise SystemExit("OrionHipSetDevice failed")
    dump(prefix + "_lib_first.txt")
    import torch  # noqa: F401  (no kernel launched)
    dump(prefix + "_after_torch.txt")
    rt = sorted({ln.split()[-1] for ln in open(prefix + "_after_torch.txt") if "libamdhip64" in ln})
    print("HIP runtimes mapped:", rt, flush=True)


if __name__ == "__main__":
    main()
