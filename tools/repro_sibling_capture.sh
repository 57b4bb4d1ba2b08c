#!/bin/bash
# Reproducer of the HIP 7.2 host crash the capture rules guard against
# (dis_plan.h R5; the r05 SIGSEGV). Builds, from a copy of this
# tree in /tmp, a variant library whose batch plan adds one barrier between the
# sub-batch streams after stage 3 (level 4 at 1080p MEDIUM): every sub-batch
# stream records an event and waits on the others' -- sibling edges -- and the
# copy's capture check is switched off so the plan reaches the runtime.
#   CPU:  tools/repro_sibling_capture.sh build   -> disflow/libdis_hip_sibling.so
#   GPU:  python3 tools/ab.py <that lib>:graphs=0 --rounds 1 --steps 2   (eager: runs)
#         python3 tools/ab.py <that lib> --rounds 1 --steps 2            (graph: SIGSEGV
#         inside hipStreamEndCapture, r06)
# (`own` events: EVENTS=own uses separate barrier events instead of the join
# events -- it crashes the same way.)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/dis_sibling_variant
rm -rf $T && mkdir -p $T
cp -r $R/optical-flow-using-dense-inverse-search_amd/csrc $R/optical-flow-using-dense-inverse-search_amd/Makefile $T/
cd $T
python3 - "${EVENTS:-join}" <<'EOF'
import sys
own = sys.argv[1] == "own"
p = "csrc/dis_plan.cpp"
s = open(p).read()
old = """    for (int t = 0; t < nstages; ++t)
        for (int k = 0; k < S; ++k) ops.push_back({kOpWork, 1 + k, -1, t});"""
e = "1 + S + " if own else "1 + "
new = """    for (int t = 0; t < nstages; ++t) {
        for (int k = 0; k < S; ++k) ops.push_back({kOpWork, 1 + k, -1, t});
        if (t == 3) {
            for (int k = 0; k < S; ++k) ops.push_back({kOpRecord, 1 + k, %sk, -1});
            for (int k = 0; k < S; ++k)
                for (int j = 0; j < S; ++j)
                    if (j != k) ops.push_back({kOpWait, 1 + k, %sj, -1});
        }
    }""" % (e, e)
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
p = "csrc/dis_runtime.hip"
s = open(p).read()
old = """        if (!why.empty()) return fail(DIS_ERR_INTERNAL, "batch stream plan cannot be captured: " + why);"""
assert old in s
s = s.replace(old, """        (void)why;  // reproducer: the check is off""")
if own:
    s = s.replace("""    auto event_of = [&](int e) { return e == 0 ? c->fork : c->join[e - 1]; };""",
                  """    auto event_of = [&](int e) { return e == 0 ? c->fork : (e <= S ? c->join[e - 1] : c->bar[e - 1 - S]); };""")
    s = s.replace("""    hipEvent_t join[kMaxSub] = {};""", """    hipEvent_t join[kMaxSub] = {};
    hipEvent_t bar[kMaxSub] = {};""")
    s = s.replace("""        ok = hipEventCreateWithFlags(&c->join[k], hipEventDisableTiming) == hipSuccess;""",
                  """        ok = hipEventCreateWithFlags(&c->join[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->bar[k], hipEventDisableTiming) == hipSuccess;""")
open(p, "w").write(s)
EOF
make -s -j8 ROOT=$R BUILD=$T/build LIB=$R/optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_sibling.so \
    $R/optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_sibling.so 2>&1 | grep -v hip-link || true
echo "built optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_sibling.so"
