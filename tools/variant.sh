#!/bin/bash
# Build a variant of libonebit_hip.so with one source recompiled under extra flags:
#   bash tools/variant.sh NAME SRC.hip "-DFOO=1 ..."  ->  exp/NAME.so
# (load it with ONEBIT_HIP_LIB=exp/NAME.so; the rest of the objects come from csrc/build)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/cmu-11785-idl-1.58bit-asr_amd/csrc
NAME=$1; SRC=$2; FLAGS=$3
make -s -C $C >/dev/null
mkdir -p $R/exp/obj
OBJ=$R/exp/obj/$NAME.${SRC%.hip}.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $FLAGS \
  -I$R/include -c $C/$SRC -o $OBJ
OBJS=$(ls $C/build/*.o | grep -v "/${SRC%.hip}.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $OBJ -o $R/exp/$NAME.so
echo "built exp/$NAME.so"
