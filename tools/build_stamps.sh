#!/bin/bash
# Diagnostic variant of libaimx.so with hop_rows.hip's phase stamps (tools/hop_stamps.py).
set -e
cd "$(dirname "$0")/../aimnet-x2d_amd/csrc"
make -j8 >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DAIMX_HOPR_STAMPS \
  -c hop_rows.hip -o /tmp/hop_rows_stamps.o
mkdir -p ../lib_stamps
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib_stamps/libaimx.so $(ls ../build/*.o | grep -v hop_rows) \
  /tmp/hop_rows_stamps.o -ldl
