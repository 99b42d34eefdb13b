#!/bin/bash
# usage: tools_resources.sh file.hip  -> kernel name, VGPRs, scratch, occupancy
cd /root/repo/statecatcher_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/root/repo/include -I. -c $1 -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: //; s/ \[-Rpass.*//' | paste - - - - | awk -F'\t' '{printf "%-70s %s | %s | %s\n", substr($1,16), $2, $3, $4}'
