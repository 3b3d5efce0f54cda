"""Build timing-only NTT variants of liborion_hip.so (never shipped).

Usage: python tools/build_ablation.py [name=FLAGS ...]
  default: abl1..abl3 (NTT_ABLATE bits: 1 no butterflies, 2 no exchanges)
  e.g.     python tools/build_ablation.py coal="-DNTT_FWD_COAL=1"
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd import build  # noqa: E402

variants = {f"abl{k}": [f"-DNTT_ABLATE={k}"] for k in (1, 2, 3)}
if len(sys.argv) > 1:
    variants = {a.split("=", 1)[0]: a.split("=", 1)[1].split() for a in sys.argv[1:]}
for name, flags in variants.items():
    out = build.build(extra_flags=flags, lib=os.path.join(build.BUILD, f"liborion_hip_{name}.so"),
                      build_dir=os.path.join(build.BUILD, name))
    print(out)
