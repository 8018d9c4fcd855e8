#!/bin/bash
# round-6 working call (overwritten per call): the odd-width hop with gathered units from global
# memory (AIMX_HOPU_VG 0 / 1 / 2) — bit-exact tests, c5 / c4 hop rooflines, c5 step
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python3 -u -m pytest -q --timeout 200 --timeout-method thread"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
tools/gpu_steps.sh \
 "600 r6f/tests.log $T -x tests/test_gpu_hop_rows.py tests/test_gpu_parity.py -k 'hop'" \
 "200 r6f/roof_c5_vg0.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=0 python3 bench.py --config c5 --roofline-only" \
 "200 r6f/roof_c5_vg1.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=1 python3 bench.py --config c5 --roofline-only" \
 "200 r6f/roof_c5_vg2.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=2 python3 bench.py --config c5 --roofline-only" \
 "200 r6f/roof_c4_vg0.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=0 python3 bench.py --config c4 --roofline-only" \
 "200 r6f/roof_c4_vg1.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=1 python3 bench.py --config c4 --roofline-only" \
 "200 r6f/roof_c4_vg2.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=2 python3 bench.py --config c4 --roofline-only" \
 "300 r6f/c5_vg2.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=2 python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6f/c5_vg0.log AIMX_LIB_PATH=$TL AIMX_HOPU_VG=0 python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline"
