#!/bin/bash
# Build experimental librrt_hip variants (block size x launch-bounds waves) into variants/.
cd "$(dirname "$0")/.."
mkdir -p variants
for cfg in "$@"; do
  b=${cfg%x*}; w=${cfg#*x}
  out=variants/b${b}w${w}
  mkdir -p $out
  make -s -C rustraytrace_amd/csrc OUT=../../$out CXXFLAGS_EXTRA="-DRRT_BLOCK=$b -DRRT_WAVES=$w" ../../$out/librrt_hip.so || exit 1
done
