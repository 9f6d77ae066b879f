#!/bin/bash
# Builds an experimental libtrainer variant with extra HIP defines into variants/ (gitignored):
#   tools/build_variant.sh NAME "-DSHRED_DELTA_LDS=512 ..."
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=$2
OUT=$HERE/../variants/$NAME
mkdir -p "$OUT"
make -s -C "$HERE" >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-parameter -I"$HERE/../include" \
  -munsafe-fp-atomics $DEFS -c "$HERE/csrc/hip/bpe_device.hip" -o "$OUT/bpe_device.o"
HOST="corpus selector tiles engine trainer dist unigram_stubs"
OBJS=""; for h in $HOST; do OBJS="$OBJS $HERE/build/$h.o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$HERE/../variants/libtrainer_$NAME.so" $OBJS "$OUT/bpe_device.o" \
  -L/opt/rocm/lib -lrccl -lamdhip64 -pthread -Wl,-rpath,/opt/rocm/lib
echo "$HERE/../variants/libtrainer_$NAME.so"
