#!/bin/bash
# Build a variant copy of the package under abvar/<tag>/ (CPU side, for same-box A/Bs): one
# kernel TU recompiled with extra hipcc flags, linked with the other objects of build/native.
# usage: tools/build_variant.sh <tag> <file.hip> <extra flags...>
set -e
cd "$(dirname "$0")/.."
tag=$1; src=$2; shift 2
out=abvar/$tag
rm -rf "$out"; mkdir -p "$out"
cp -r smdistributed_modelparallel_amd "$out/"; rm -rf "$out/smdistributed_modelparallel_amd/csrc"; find "$out" -name __pycache__ -prune -exec rm -rf {} +
cp bench.py "$out/"; cp -r configs "$out/"
abi=$(python3 -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
tlib=$(python3 -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
kd=smdistributed_modelparallel_amd/csrc/kernels
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
  -D_GLIBCXX_USE_CXX11_ABI=$abi -munsafe-fp-atomics -Wno-unused-result -I$kd "$@" -c $kd/$src -o "$out/$src.o"
objs=$(ls build/native/kernels/*.o | grep -v "/$src.o$")
so=$(ls smdistributed_modelparallel_amd/_C*.so | xargs -n1 basename)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/smdistributed_modelparallel_amd/$so" $objs "$out/$src.o" \
  -L$tlib -Wl,-rpath,$tlib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64
rm -f "$out/$src.o"
echo "built $out"
