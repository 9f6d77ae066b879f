#!/bin/bash
# Builds an experimental libtrainer variant with extra HIP defines into variants/ (gitignored),
# linked like the Makefile's library; select it with SHREDWORD_LIB=variants/libtrainer_NAME.so:
#   tools/build_variant.sh NAME "-DSHRED_WL_STAMPS ..."
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=$2
OUT=$HERE/../variants/$NAME
mkdir -p "$OUT"
make -s -C "$HERE" >/dev/null
HIPOBJS=""
for f in bpe_device load_device encode_device word_loop; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-parameter -I"$HERE/../include" \
    -munsafe-fp-atomics $DEFS -c "$HERE/csrc/hip/$f.hip" -o "$OUT/$f.o" &
  HIPOBJS="$HIPOBJS $OUT/$f.o"
done
wait
OBJS=""; for h in corpus selector tiles engine trainer dist unigram_stubs encoder; do OBJS="$OBJS $HERE/build/$h.o"; done
g++ -shared -fPIC -o "$HERE/../variants/libtrainer_$NAME.so" $OBJS $HIPOBJS -L"$HERE/build/stub" -Wl,--no-as-needed \
  -lamdhip64 -lhsa-runtime64 -lrocprofiler-register -lamd_comgr -lnuma -ldl -pthread -Wl,-rpath,/opt/rocm/lib
echo "$HERE/../variants/libtrainer_$NAME.so"
