#!/bin/bash
# Build an A/B variant of the extension: recompile some csrc/*.hip files with extra -D flags and
# link them with the other objects of the current build into xdot/_C_<name>.so (load it with
# XDOT_EXT_PATH=xdot/_C_<name>.so).  usage: build_variant.sh NAME "A.hip B.hip" "-DFOO -DBAR"
set -e
NAME=$1; SRCS=$2; DEFS=$3
python -m xdot.build > /dev/null
B=build/variant_$NAME
mkdir -p $B
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
TLIB=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
for SRC in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I csrc -fno-slp-vectorize -D__HIP_PLATFORM_AMD__=1 \
    -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$ABI -Wno-unused-result -Wno-unused-variable $DEFS -c csrc/$SRC -o $B/$SRC.o &
done
wait
OBJS=""
for o in build/xdot/*.o; do
  base=$(basename $o .o)
  if [ -f "$B/$base.o" ] && [[ " $SRCS " == *" $base "* ]]; then OBJS="$OBJS $B/$base.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o xdot/_C_$NAME.so $OBJS -L $TLIB -Wl,-rpath,$TLIB -lc10 -lc10_hip \
  -ltorch -ltorch_cpu -ltorch_hip -lamdhip64 -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
echo xdot/_C_$NAME.so
