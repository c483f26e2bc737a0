#!/usr/bin/env bash
# Per-kernel register / scratch / occupancy summary of one HIP source (device compile only).
#   tools/kres.sh <file.hip> [name-filter]
f="$1"; filt="${2:-.}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
    --cuda-device-only -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed "s/ \[-Rpass-analysis=kernel-resource-usage\]//" | awk '/Function Name:/{n=$NF} /VGPRs:/{v=$NF} /AGPRs:/{a=$NF} /ScratchSize/{s=$NF} /Occupancy/{o=$NF; print n, "vgpr="v, "agpr="a, "scratch="s, "occ="o}' |
  grep -E "$filt" | sed 's/_ZN6hipann//' | cut -c1-140
