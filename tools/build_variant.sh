#!/bin/bash
# Development A/B builds: tools/build_variant.sh NAME SOURCE "-DFLAG=V ..." ->
# tools/variants/libspecenh_NAME.so (every other object from the in-tree build); load it
# with SPECENH_LIB=$PWD/tools/variants/libspecenh_NAME.so. SOURCE may be a path (e.g. an older
# revision of a csrc file written elsewhere); it replaces the csrc object of the same basename.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; DEFS=$3
case $SRC in */*) SRCP=$SRC;; *) SRCP=$R/spectrogram-enhancement_amd/csrc/$SRC;; esac
OBJ=$R/spectrogram-enhancement_amd/build/obj
OUT=$R/tools/variants
mkdir -p $OUT
python3 $R/spectrogram-enhancement_amd/build.py > /dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/spectrogram-enhancement_amd/csrc \
  -Xclang -target-feature -Xclang -packed-fp32-ops $DEFS -c $SRCP -o $OUT/$NAME.o
OBJS=$(ls $OBJ/*.o | grep -v "/$(basename $SRC).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libspecenh_$NAME.so $OBJS $OUT/$NAME.o
echo $OUT/libspecenh_$NAME.so
