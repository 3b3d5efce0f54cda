"""Build liborion_hip.so in-tree for gfx950 (hipcc, no JIT cache)."""
import fcntl
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "liborion_hip.so")
ARCH = os.environ.get("ORION_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: the float64 quotient of the exact basis extension and the
# encoder FFT must round exactly as written (bit parity with the CPU oracle).
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]
SOURCES = ["ntt.hip", "ntt2.hip", "ntt2s.hip", "kernels.hip", "encoder.hip", "backend.hip", "hostmath.cpp", "wire.cpp"]


def _needs(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _stamp(build_dir, recipe):
    """Rebuild everything when the compiler, the arch or any flag changed since
    the objects in build_dir were made (mtimes alone miss a new -D flag)."""
    path = os.path.join(build_dir, "recipe.json")
    digest = hashlib.sha256(json.dumps(recipe, sort_keys=True).encode()).hexdigest()
    old = None
    if os.path.exists(path):
        try:
            with open(path) as f:
                old = json.load(f).get("digest")
        except ValueError:  # a stamp cut short: rebuild
            old = None
    return path, digest, old != digest


def build(verbose=False, extra_flags=(), lib=LIB, build_dir=BUILD):
    """Compile liborion_hip.so (extra_flags/lib/build_dir: timing-only variants).
    Concurrent callers (pytest -n workers) serialise on a lock in build_dir."""
    os.makedirs(build_dir, exist_ok=True)
    with open(os.path.join(build_dir, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return _build(verbose, extra_flags, lib, build_dir)


def _build(verbose, extra_flags, lib, build_dir):
    BUILD_, LIB_ = build_dir, lib
    recipe = {"hipcc": HIPCC, "arch": ARCH, "flags": FLAGS + list(extra_flags), "sources": SOURCES}
    stamp, digest, changed = _stamp(BUILD_, recipe)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "orion_hip.h"))
    headers.append(os.path.abspath(__file__))
    objs, jobs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD_, src + ".o")
        objs.append(obj)
        if changed or _needs(obj, [path] + headers):
            cmd = [HIPCC] + FLAGS + list(extra_flags) + ["-c", path, "-o", obj]
            if src.endswith(".hip"):
                cmd.insert(1, f"--offload-arch={ARCH}")
            jobs.append(cmd)

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("compile failed: " + " ".join(cmd) + "\n" + r.stderr)
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)

    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(run, jobs))
    if jobs or changed or not os.path.exists(LIB_):
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_] + objs)
    with open(stamp + ".tmp", "w") as f:
        json.dump({"digest": digest, "recipe": recipe}, f, indent=1)
    os.replace(stamp + ".tmp", stamp)
    return LIB_


if __name__ == "__main__":
    print(build(verbose=True))
