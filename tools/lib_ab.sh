#!/bin/bash
# Interleaved A/B of whole library builds on one box: bash tools/lib_ab.sh TOOL ARGS -- LIB...
# (LIB "main" = the in-tree library; others: tools/variants/libspecenh_NAME.so). ROUNDS rounds (default 2).
TOOL=$1; shift
ARGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARGS+=("$1"); shift; done
shift
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for L in "$@"; do
    if [ "$L" = main ]; then
      echo "== $L (round $rnd)"; timeout -k 10 120 python $TOOL "${ARGS[@]}" || exit 1
    else
      echo "== $L (round $rnd)"; SPECENH_LIB=$PWD/tools/variants/libspecenh_$L.so timeout -k 10 120 python $TOOL "${ARGS[@]}" || exit 1
    fi
  done
done
