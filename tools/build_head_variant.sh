#!/bin/bash
# The r06 coarse-head experiment (verdict r05 item 1), kept
# reproducible outside the product: applies tools/patches/r06_coarse_head.patch
# (k_search8_head: levels 6..4 of a sub-batch in one launch, ticket-ordered
# blocks, write-through hand-off of each level's patch displacements) to a copy
# of this tree in /tmp and builds it as a variant library; STAMPS=1 adds
# per-workgroup s_memrealtime stamps (tools/patches/r06_head_stamps.py) read by
# tools/head_probe.py.
#   CPU:  tools/build_head_variant.sh            -> disflow/libdis_hip_head.so
#         STAMPS=1 tools/build_head_variant.sh   -> disflow/libdis_hip_headts.so
#   GPU:  tools/gpu/session.sh ab=libdis_hip.so,libdis_hip_head.so
#         python3 tools/head_probe.py optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_headts.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/optical-flow-using-dense-inverse-search_amd
NAME=head; [ "${STAMPS:-0}" = 1 ] && NAME=headts
T=/tmp/dis_${NAME}_variant
rm -rf $T && mkdir -p $T/optical-flow-using-dense-inverse-search_amd
cp -r $P/csrc $P/Makefile $T/optical-flow-using-dense-inverse-search_amd/
cd $T && patch -s -p1 < $R/tools/patches/r06_coarse_head.patch
cd $T/optical-flow-using-dense-inverse-search_amd
[ "$NAME" = headts ] && python3 $R/tools/patches/r06_head_stamps.py
make -s -j8 ROOT=$R BUILD=$T/build LIB=$P/disflow/libdis_hip_$NAME.so $P/disflow/libdis_hip_$NAME.so 2>&1 | grep -v hip-link || true
echo "built $P/disflow/libdis_hip_$NAME.so"
