#!/bin/bash
# Build experimental variants of one translation unit into leastereo_amd/var_<name>.so
# (selected at run time with LEASTEREO_HIP_LIB).  usage: build_variants.sh UNIT name:"flags" ...
# The LEA_EXP_* ablation switches are not in the product sources: the variants compile a
# copy of leastereo_amd/csrc with tools/ablation/*.patch applied (tools/ablation.py).
set -eu
cd "$(dirname "$0")/.."
make -s -j8
UNIT=$1; shift
VSRC=build/var/src
rm -rf $VSRC && mkdir -p $VSRC && cp leastereo_amd/csrc/*.hip leastereo_amd/csrc/*.h $VSRC/
python3 tools/ablation.py apply $VSRC
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build/var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Iinclude \
    -I$VSRC -munsafe-fp-atomics -DLEA_ABLATION_BUILD $flags -c $VSRC/$UNIT.hip -o build/var/$name/$UNIT.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  objs=$(ls build/obj/*.o | grep -v "/$UNIT.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o leastereo_amd/var_$name.so $objs build/var/$name/$UNIT.o
done
ls -la leastereo_amd/var_*.so
