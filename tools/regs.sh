#!/bin/bash
# Print VGPR / SGPR / scratch / occupancy of the simulate kernels (compile-time resource usage).
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm -fPIC -shared -I include "$@" -o /tmp/regs.so \
  topotrafficrl_amd/csrc/ttrl_mi355x.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
  | awk '/Function Name/{n=$NF; sub(/\[.*/,"",n); name=$0; sub(/.*Function Name: /,"",name); sub(/ \[.*/,"",name)}
         /VGPRs:/{v=$0; sub(/.*VGPRs: /,"",v); sub(/ .*/,"",v)}
         /AGPRs:/{a=$0; sub(/.*AGPRs: /,"",a); sub(/ .*/,"",a)}
         /ScratchSize/{sc=$0; sub(/.*lane\]: /,"",sc); sub(/ .*/,"",sc)}
         /Occupancy/{o=$0; sub(/.*Occupancy \[waves\/SIMD\]: /,"",o); sub(/ .*/,"",o); printf "%-70s vgpr=%s agpr=%s scratch=%s occ=%s\n", substr(name,1,70), v, a, sc, o}' \
  | grep -E "simulate|${FILTER:-simulate}"
