#!/bin/bash
# Capture MI355X telemetry sources as test fixtures: amd-smi / rocm-smi JSON and the AMD sysfs
# files the node telemetry reader uses (values only; nothing is written outside gpurun_out/).
set -o pipefail
out=gpurun_out/telemetry
mkdir -p $out/sysfs
timeout -k 5 60 amd-smi metric --json > $out/amd_smi_metric.json 2> $out/amd_smi_metric.err || echo "amd-smi metric rc=$?"
timeout -k 5 60 amd-smi static --asic --json > $out/amd_smi_static.json 2> $out/amd_smi_static.err || echo "amd-smi static rc=$?"
timeout -k 5 60 rocm-smi --showuse --showmeminfo vram --showpower --showtemp --json > $out/rocm_smi.json 2> $out/rocm_smi.err || echo "rocm-smi rc=$?"
for card in /sys/class/drm/card[0-9]*; do
  case "$card" in *-*) continue;; esac
  d=$card/device
  [ -f $d/mem_info_vram_total ] || continue
  c=$(basename $card)
  mkdir -p $out/sysfs/$c/device/hwmon
  for f in mem_info_vram_total mem_info_vram_used gpu_busy_percent pp_dpm_sclk product_name unique_id; do
    [ -r $d/$f ] && cat $d/$f > $out/sysfs/$c/device/$f 2>/dev/null
  done
  for h in $d/hwmon/hwmon*; do
    hn=$(basename $h); mkdir -p $out/sysfs/$c/device/hwmon/$hn
    for f in name power1_average power1_input temp1_input temp1_label temp2_input temp2_label temp3_input temp3_label; do
      [ -r $h/$f ] && cat $h/$f > $out/sysfs/$c/device/hwmon/$hn/$f 2>/dev/null
    done
  done
  echo "captured $c"
done
ls -R $out | head -50
