#!/bin/bash
# Probe the GPU box's sysfs/procfs layout that the exporter's KFD/drm/cgroup readers depend on.
# Usage (GPU box): bash tools/probe_host.sh > gpurun_out/probe_host.txt 2>&1
set +e
echo "== id"; id; uname -r; nproc
echo "== /proc/self/cgroup"; cat /proc/self/cgroup
echo "== /proc/1/cgroup"; cat /proc/1/cgroup 2>&1 | head
echo "== mount cgroup"; grep cgroup /proc/self/mountinfo | head
echo "== kfd topology nodes"
for n in /sys/class/kfd/kfd/topology/nodes/*; do
  echo "-- $n gpu_id=$(cat $n/gpu_id 2>/dev/null) name=$(cat $n/name 2>/dev/null)"
  grep -E "^(location_id|domain|drm_render_minor|unique_id|simd_count|array_count|cu_per_simd_array|max_engine_clk_fcompute|num_xcc|local_mem_size|device_id|gfx_target_version|num_sdma_engines|hive_id)" $n/properties 2>/dev/null
done
echo "== kfd proc"; ls -la /sys/class/kfd/kfd/proc/ 2>&1 | head -20
for p in /sys/class/kfd/kfd/proc/*; do echo "-- $p"; ls -la $p 2>&1 | head -30; done 2>/dev/null | head -60
echo "== drm"; ls /sys/class/drm/
for c in /sys/class/drm/card*; do
  [ -e "$c/device/gpu_metrics" ] || continue
  echo "-- $c"
  ls $c/device/ | tr '\n' ' '; echo
  for f in gpu_busy_percent mem_busy_percent mem_info_vram_used mem_info_vram_total unique_id current_link_speed current_link_width; do
    echo "$f=$(cat $c/device/$f 2>&1)"
  done
  ls -la $c/device/gpu_metrics
  xxd $c/device/gpu_metrics | head -4
  echo "hwmon:"; for h in $c/device/hwmon/*; do ls $h | tr '\n' ' '; echo; for f in $h/power1_average $h/power1_input $h/temp1_input $h/temp2_input $h/temp3_input $h/temp1_label $h/temp2_label $h/temp3_label $h/energy1_input; do [ -e $f ] && echo "$f=$(cat $f 2>&1)"; done; done
  break
done
echo "== uevent of render nodes"; for r in /sys/class/drm/renderD*; do echo "$r $(cat $r/device/uevent 2>/dev/null | grep PCI_SLOT_NAME)"; done | head
echo "== /dev"; ls -la /dev/kfd /dev/dri/ 2>&1 | head -20
echo "== rocm-smi"; timeout 30 rocm-smi --showuse --showmeminfo vram --showpower --showtemp 2>&1 | head -40
echo "== amd-smi"; timeout 30 amd-smi metric -g 0 2>&1 | head -120
echo "== rocprofv3 -L (counters gfx950)"; timeout 60 rocprofv3 -L 2>&1 | grep -E "SQ_VALU_MFMA_BUSY_CYCLES|SQ_BUSY_CYCLES|GRBM_GUI_ACTIVE|SQ_WAVES\b|SQ_LDS_IDX_ACTIVE|SQ_LDS_BANK_CONFLICT|TCC_EA0_RDREQ\b|TCC_EA0_WRREQ\b|GRBM_COUNT" | head -20
echo "== perf_event_paranoid"; cat /proc/sys/kernel/perf_event_paranoid
echo "== done"
