#!/bin/bash
# Build experimental variants of one translation unit into leastereo_amd/var_<name>.so
# (selected at run time with LEASTEREO_HIP_LIB).  usage: build_variants.sh UNIT name:"flags" ...
set -eu
cd "$(dirname "$0")/.."
make -s -j8
UNIT=$1; shift
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build/var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Iinclude \
    -Ileastereo_amd/csrc -munsafe-fp-atomics -DLEA_ABLATION_BUILD $flags -c leastereo_amd/csrc/$UNIT.hip -o build/var/$name/$UNIT.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  objs=$(ls build/obj/*.o | grep -v "/$UNIT.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o leastereo_amd/var_$name.so $objs build/var/$name/$UNIT.o
done
ls -la leastereo_amd/var_*.so
