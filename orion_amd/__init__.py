"""MI355X (gfx950) HIP backend for Orion's RNS-CKKS ciphertext arithmetic.

Product path: orion_amd/csrc (HIP kernels + C-ABI, built into
liborion_hip.so) and orion_amd/backend.py (HipLibrary, the drop-in for the
reference's LattigoLibrary).  There is no CPU fallback.
"""
__all__ = ["backend", "replay", "build"]
