#!/bin/bash
# probe libraries of the diagonal-tile kernel alone (csrc/chol.hip + lcq_common.hip) with the
# s_memtime stage stamps (-DLCQ_CHOL_PROF) for scripts/chol_tile_prof2.py: the product
# (hardware v_sqrt / v_rcp: libchol_prof2.so) and IEEE sqrt / division (libchol_prof2_ieee.so)
set -e
cd "$(dirname "$0")/.."
C=lightcompress_amd/csrc
for v in "libchol_prof2.so:" "libchol_prof2_ieee.so:-DLCQ_PROBE_CHOL_IEEE_RSQ=1"; do
  out=${v%%:*}; def=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -DLCQ_CHOL_PROF $def \
    $C/chol.hip $C/lcq_common.hip -o scripts/_lib/$out
done
echo built
