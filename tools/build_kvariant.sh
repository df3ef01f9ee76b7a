#!/bin/bash
# Build an A/B copy of the kernel extension: the given kernel TUs recompiled with extra hipcc
# flags (e.g. -D macros an experiment adds), linked with the in-tree objects of every
# other TU, written to abtest/_C_<tag>.so (abtest/ travels with gpurun; time it with
# tools/kvariant_time.py or tools/attn_time.py <so>).  A TU's own in-tree flags
# (_build._TU_FLAGS, e.g. the dQ TU's -fno-slp-vectorize) are kept.
# usage: tools/build_kvariant.sh <tag> <file.hip>[,<file2.hip>...] <flags...>
set -e
cd "$(dirname "$0")/.."
tag=$1; srcs=$2; shift 2
mkdir -p abtest build/kvariant
abi=$(python3 -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
tlib=$(python3 -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
kd=smdistributed_modelparallel_amd/csrc/kernels
objs=$(ls build/native/kernels/*.o)
vobjs=""
for src in ${srcs//,/ }; do
  tuf=$(python3 -c "import sys; sys.path.insert(0, '.'); from smdistributed_modelparallel_amd._build import _TU_FLAGS; print(' '.join(_TU_FLAGS.get('$src', [])))")
  obj=build/kvariant/${tag}_$src.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
    -D_GLIBCXX_USE_CXX11_ABI=$abi -munsafe-fp-atomics -Wno-unused-result -I$kd $tuf "$@" -c $kd/$src -o $obj &
  objs=$(echo "$objs" | grep -v "/$src.o$")
  vobjs="$vobjs $obj"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o abtest/_C_$tag.so $objs $vobjs \
  -L$tlib -Wl,-rpath,$tlib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64
echo "built abtest/_C_$tag.so"
