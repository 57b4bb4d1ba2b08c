#!/bin/bash
# One GPU session from named steps (replaces the r03 one-off session scripts):
#   tools/gpu/session.sh <step> [<step> ...]
# Steps (each under its own time limit; a crash, abort or timeout ends the
# session, a plain test / A/B failure too):
#   tests[=<pytest -k expr>]     GPU suite (or a subset), one process
#   ab=<lib[:opts]>,<lib>,...    interleaved whole-step A/B (tools/ab.py, one process)
#   abspawn=<lib>,<lib>,...      the same, one process per variant and round (4 rounds)
#   levels=<lib>,<lib>,...       per-kernel one-stream durations (rocprof kernel trace)
#   pmc=<lib>                    SQ counters of the top kernels (tools/gpu/pmc_sq.sh; CTRS= to override)
#   bench                        bench.py default line
#   smoke                        __graft_entry__.smoke()
#   tool=<name> [args]           a built tools/ binary (e.g. tool=issue_mix)
#   py=<script> [args]           a python script of the repo (e.g. py="tools/bench_configs.py --configs colour")
#   prof=<script> [args]         the same under rocprofv3 --kernel-trace --stats: top kernels by total time
# Libraries are paths relative to the package's disflow/ (e.g. libdis_hip_x.so);
# build variants first on the CPU: tools/build_variants.sh name:"-DFLAG=1".
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
libs() { local out=(); IFS=, read -ra a <<< "$1"; for v in "${a[@]}"; do out+=("$D/$v"); done; echo "${out[@]}"; }
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-12}
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
n=0
for s in "$@"; do
  n=$((n+1)); k=${s%%=*}; v=${s#*=}
  case $k in
    tests) if [ "$s" = tests ]; then run s${n}_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
           else run s${n}_tests 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$v"; fi ;;
    ab) run s${n}_ab 600 python3 tools/ab.py $(libs "$v") --rounds 8 --steps 10 ;;
    abspawn) run s${n}_abspawn 900 python3 tools/ab.py --spawn 4 --rounds 3 --steps 10 $(libs "$v") ;;
    levels) run s${n}_levels 600 bash tools/gpu/levels.sh $(libs "$v") ;;
    pmc) run s${n}_pmc 300 bash tools/gpu/pmc_sq.sh $(libs "$v") ;;
    bench) run s${n}_bench 400 python bench.py ;;
    smoke) run s${n}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tool) run s${n}_$(echo "$v" | cut -d' ' -f1) 300 ./tools/$v ;;
    py) run s${n}_$(basename "$(echo "$v" | cut -d' ' -f1)" .py) 600 python3 $v ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/gpurun_out/prof_s$n" -o run -- python3 "$GRAFT_REPO_ROOT"/$v) > gpurun_out/s${n}_prof.log 2>&1
          rc=$?; echo "== s${n}_prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s${n}_prof.log; exit $rc; }
          python3 - gpurun_out/prof_s$n/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f"  {r['Name'][:60]:60s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs']) / 1e3:9.2f} us  total {float(r['TotalDurationNs']) / 1e6:9.3f} ms")
PY
          ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
