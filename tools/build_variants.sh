#!/bin/bash
# Build experimental librrt_hip variants into variants/<name>/.
#   BxW            block size x launch-bounds waves, e.g. 512x6
#   name:FLAGS     arbitrary extra compile flags, e.g. "pt1:-DRRT_PHASE_TIMING=1"
# F64_FLAGS (env) goes to the f64 kernel object only.
cd "$(dirname "$0")/.."
mkdir -p variants
for cfg in "$@"; do
  if [[ $cfg == *:* ]]; then
    name=${cfg%%:*}; flags=${cfg#*:}
  else
    b=${cfg%x*}; w=${cfg#*x}
    name=b${b}w${w}; flags="-DRRT_BLOCK=$b -DRRT_WAVES=$w"
  fi
  out=variants/$name
  rm -rf $out && mkdir -p $out
  make -s -C rustraytrace_amd/csrc OUT=../../$out CXXFLAGS_EXTRA="$flags" F64_FLAGS="${F64_FLAGS:-}" ../../$out/librrt_hip.so || exit 1
done
