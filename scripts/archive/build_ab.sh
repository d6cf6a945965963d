#!/bin/bash
# Build the A side of an A/B: recompile ONE csrc/*.hip file as it is at git revision REV and link
# it with the other objects of the current build into xdot/_C_<name>.so (load it with
# XDOT_EXT_PATH=xdot/_C_<name>.so).  usage: build_ab.sh NAME REV SOURCE.hip
set -e
NAME=$1; REV=$2; SRC=$3
python -m xdot.build > /dev/null
B=build/ab_$NAME
mkdir -p $B
git show $REV:csrc/$SRC > $B/$SRC
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
TLIB=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I csrc -fno-slp-vectorize -D__HIP_PLATFORM_AMD__=1 \
  -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$ABI -Wno-unused-result -Wno-unused-variable -c $B/$SRC -o $B/$SRC.o
OBJS=""
for o in build/xdot/*.o; do
  if [ "$(basename $o)" == "$SRC.o" ]; then OBJS="$OBJS $B/$SRC.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o xdot/_C_$NAME.so $OBJS -L $TLIB -Wl,-rpath,$TLIB -lc10 -lc10_hip \
  -ltorch -ltorch_cpu -ltorch_hip -lamdhip64 -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
echo xdot/_C_$NAME.so
