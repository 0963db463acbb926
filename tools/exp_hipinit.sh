#!/bin/bash
# HIP start-up in fresh processes under environment variants (tools/exp_hipinit.cpp); 5 runs each.
cd "$GRAFT_REPO_ROOT" || exit 1
echo "# env:"; env | grep -E "VISIBLE|^HSA_|^HIP_|^ROCR|^GPU_|^AMD_" | sort
echo "# kfd nodes: $(ls /sys/class/kfd/kfd/topology/nodes | wc -l); render nodes: $(ls /dev/dri | grep -c render)"
for v in "-" "ROCR_VISIBLE_DEVICES=0" "HIP_VISIBLE_DEVICES=0" "GPU_MAX_HW_QUEUES=8" "HSA_ENABLE_SDMA=0" \
         "HSA_ENABLE_INTERRUPT=0" "ROCR_VISIBLE_DEVICES=0,GPU_MAX_HW_QUEUES=8" "-"; do
  for i in 1 2 3 4 5; do
    if [ "$v" = "-" ]; then timeout -k 5 60 ./tools/exp_hipinit.bin; else env ${v//,/ } timeout -k 5 60 ./tools/exp_hipinit.bin; fi | sed "s/^/$v /"
  done
done
