"""GPU: replay the reference frontend's ResNet-20 (CIFAR-10) op stream
(tests/golden/resnet20_n13_*, configs/resnet.yml parameters, 42 bootstraps,
138 polynomial evaluations) and compare the decrypted logits with the
cleartext model."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.replay import OrionStream  # noqa: E402


def main():
    B = int(os.environ.get("BATCH", 1))
    st = OrionStream("resnet20_n13", seed=3)
    t0 = time.perf_counter()
    st.keygen()
    st.compile()
    st.lib.OrionHipSynchronize()
    print("keygen+compile", round(time.perf_counter() - t0, 1), "s", flush=True)
    img = st.reference_input()
    ct = st.encrypt_batch(np.repeat(img, B, axis=0))
    t0 = time.perf_counter()
    out = st.forward(ct)
    st.lib.OrionHipSynchronize()
    dt = time.perf_counter() - t0
    res = st.decrypt_output(out)
    exp = st.arrays["expected_output"].reshape(-1)
    print("forward", round(dt, 2), "s for", B, "images; logits", np.round(res[0], 4), flush=True)
    print("expected", np.round(exp, 4), "max abs err", float(np.abs(res[0] - exp).max()),
          "argmax match", int(np.argmax(res[0]) == np.argmax(exp)), flush=True)


if __name__ == "__main__":
    main()
