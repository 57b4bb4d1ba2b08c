#!/bin/bash
# Read-only probe of what the box exposes for clock / power sampling (sysfs
# hwmon, gpu_metrics, amd-smi) -- which source bench.py can sample cheaply.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{
for d in /sys/class/drm/card*/device; do
  [ -e "$d/gpu_metrics" ] || continue
  echo "== $d -> $(readlink -f $d)"
  ls "$d/hwmon/" 2>/dev/null
  for h in "$d"/hwmon/hwmon*; do
    for f in "$h"/freq*_input "$h"/freq*_label "$h"/power*_average "$h"/power*_input "$h"/power*_cap "$h"/temp*_input "$h"/in*_input; do
      [ -e "$f" ] && echo "$f = $(cat $f 2>&1)"
    done
  done
  for f in pp_dpm_sclk pp_dpm_mclk current_link_speed current_link_width; do
    [ -e "$d/$f" ] && { echo "-- $f"; cat "$d/$f" 2>&1 | head -12; }
  done
  echo "-- gpu_metrics: $(stat -c %s $d/gpu_metrics 2>&1) bytes, header $(head -c 4 $d/gpu_metrics | od -An -tu1 2>&1)"
done
echo "== amd-smi"
( time timeout 30 amd-smi metric -g 0 --power --clock --json ) 2>&1 | head -80
} > gpurun_out/boxstate.log 2>&1
python3 - <<'PY' >> gpurun_out/boxstate.log 2>&1
import torch
p = torch.cuda.get_device_properties(0)
print({k: getattr(p, k) for k in dir(p) if not k.startswith("_") and "pci" in k.lower()})
PY
tail -c 4000 gpurun_out/boxstate.log
