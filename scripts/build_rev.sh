#!/bin/bash
# Build an A/B variant whose listed csrc files come from git revision REV (the rest from the current
# build) into xdot/_C_<name>.so (load with XDOT_EXT_PATH).  usage: build_rev.sh NAME REV "A.hip B.hip"
set -e
NAME=$1; REV=$2; SRCS=$3
python -m xdot.build > /dev/null
B=build/variant_$NAME
rm -rf $B; mkdir -p $B/src
# headers from REV too (a header change is part of the variant)
for h in $(git ls-tree --name-only $REV csrc/ | grep '\.h$'); do git show $REV:$h > $B/src/$(basename $h); done
for SRC in $SRCS; do git show $REV:csrc/$SRC > $B/src/$SRC; done
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
TLIB=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
for SRC in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I $B/src -fno-slp-vectorize -D__HIP_PLATFORM_AMD__=1 \
    -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$ABI -Wno-unused-result -Wno-unused-variable -c $B/src/$SRC -o $B/$SRC.o &
done
wait
OBJS=""
for o in build/xdot/*.o; do
  base=$(basename $o .o)
  if [ -f "$B/$base.o" ]; then OBJS="$OBJS $B/$base.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o xdot/_C_$NAME.so $OBJS -L $TLIB -Wl,-rpath,$TLIB -lc10 -lc10_hip \
  -ltorch -ltorch_cpu -ltorch_hip -lamdhip64 -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
echo xdot/_C_$NAME.so
