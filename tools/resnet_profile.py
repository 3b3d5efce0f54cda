import os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd())
from orion_amd.replay import OrionStream
st = OrionStream("resnet20_n13", seed=3); st.keygen(); st.compile()
lib = st.lib
ct = st.encrypt_batch(st.reference_input())
lib.DeleteCiphertext(st.forward(ct)); lib.OrionHipSynchronize()
lib.OrionHipProfileReset(); lib.OrionHipProfile(1)
t0 = time.perf_counter(); out = st.forward(ct); lib.OrionHipSynchronize(); dt = time.perf_counter() - t0
lib.OrionHipProfile(0)
prof = lib.profile_read()
tot = sum(v["ms"] for v in prof.values()); nl = sum(v["launches"] for v in prof.values())
print("wall", round(dt, 3), "s; kernel ms", round(tot, 1), "launches", nl)
print({k: (round(v["ms"], 1), v["launches"]) for k, v in prof.items()})
