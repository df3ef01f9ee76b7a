#!/bin/bash
# Build an A/B copy of the kernel extension: one kernel TU recompiled with extra hipcc flags
# (e.g. -DSMPK_WGRAD_TK=32 -DSMPK_WGRAD_NS=4), linked with the in-tree objects of every other
# TU, written to abtest/_C_<tag>.so (abtest/ travels with gpurun; load it with
# tools/kvariant_time.py).  usage: tools/build_kvariant.sh <tag> <file.hip> <flags...>
set -e
cd "$(dirname "$0")/.."
tag=$1; src=$2; shift 2
mkdir -p abtest build/kvariant
abi=$(python3 -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
tlib=$(python3 -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
kd=smdistributed_modelparallel_amd/csrc/kernels
obj=build/kvariant/${tag}_$src.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
  -D_GLIBCXX_USE_CXX11_ABI=$abi -munsafe-fp-atomics -Wno-unused-result -I$kd "$@" -c $kd/$src -o $obj
objs=$(ls build/native/kernels/*.o | grep -v "/$src.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o abtest/_C_$tag.so $objs $obj \
  -L$tlib -Wl,-rpath,$tlib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64
echo "built abtest/_C_$tag.so"
