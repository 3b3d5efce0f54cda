"""GPU debug: replay ResNet-20 and report, per op, the max |slot| of the result
until values blow up."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.replay import OrionStream  # noqa: E402


def main():
    st = OrionStream("resnet20_n13", seed=3)
    st.keygen()
    st.compile()
    lib = st.lib
    ct = st.encrypt_batch(st.reference_input())
    log = []
    state = {"bad": 0}

    def hook(ev, h):
        if state["bad"] > 3:
            return
        pt = lib.Decrypt(h)
        v = lib.decode_f64(pt)[0]
        lib.DeletePlaintext(pt)
        m = float(np.abs(v).max())
        lv, sc = lib.GetCiphertextLevel(h), lib.GetCiphertextScaleF(h)
        log.append((len(log), ev["op"], ev["args"], lv, sc, m))
        if m > 50:
            state["bad"] += 1
            for row in log[-12:]:
                print(row, flush=True)
            print("----", flush=True)

    st.forward(ct, hook=hook)
    if state["bad"] == 0:
        print("no blow-up; last", log[-3:])


if __name__ == "__main__":
    main()
