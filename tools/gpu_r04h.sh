# r04h: lt_bsgs_kernel8 regression bisect (1848 -> 1937 us at 91f9e70): the
# baby pre-split (LT_PRESPLIT) and the split-key gadget path (LT_GADGET_W)
PARITY=0 NTT=0 BENCH=1 KPROF=1 bash tools/ab.sh r04h lib product nops nogw none
