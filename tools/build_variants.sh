#!/bin/bash
# Build A/B variant libraries next to the default one:
#   tools/build_variants.sh name:"<compiler flags>" ...
# -> optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_<name>.so
# Flags: compiler options (e.g. -mllvm scheduler switches), or -D switches of
# an uncommitted experiment in the working tree -- committed sources carry no
# compile-time variants (tests/test_no_compile_switches.py).
set -e
cd "$(dirname "$0")/../optical-flow-using-dense-inverse-search_amd"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  make -s -j8 BUILD=build_$name LIB=disflow/libdis_hip_$name.so EXTRA="-fno-slp-vectorize $flags" disflow/libdis_hip_$name.so 2>&1 | grep -v hip-link || true
done
