#!/bin/bash
# Build A/B variant libraries next to the default one:
#   tools/build_variants.sh name:"-DFLAG=1 -DOTHER=2" ...
# -> optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_<name>.so
set -e
cd "$(dirname "$0")/../optical-flow-using-dense-inverse-search_amd"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  # knock-out switches (wrong values) must be asked for explicitly (csrc/dis_experiments.h)
  case "$flags" in *DIS_EXP_*) flags="$flags -DDIS_EXPERIMENTS";; esac
  make -s -j8 BUILD=build_$name LIB=disflow/libdis_hip_$name.so EXTRA="-fno-slp-vectorize $flags" disflow/libdis_hip_$name.so 2>&1 | grep -v hip-link || true
done
