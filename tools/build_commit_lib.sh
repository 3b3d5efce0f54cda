# Build liborion_hip.so from the sources of an earlier commit (timing A/B only, never shipped)
# usage: bash tools/build_commit_lib.sh COMMIT NAME  ->  orion_amd/_build/liborion_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
C=$1; NAME=$2
D=/tmp/orion_commit_$NAME
rm -rf $D && mkdir -p $D
git archive $C orion_amd/csrc include | tar -x -C $D
OUT=orion_amd/_build/liborion_hip_$NAME.so
OBJS=""
for s in ntt.hip ntt2.hip kernels.hip encoder.hip backend.hip hostmath.cpp wire.cpp; do
  A=""; case $s in *.hip) A=--offload-arch=gfx950;; esac
  /opt/rocm/bin/hipcc $A -O3 -fPIC -std=c++17 -ffp-contract=off -w -c $D/orion_amd/csrc/$s -o $D/$s.o &
  OBJS="$OBJS $D/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS
echo $OUT
