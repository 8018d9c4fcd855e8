#!/bin/bash
# round-5 working call (overwritten per call): Adam with the clip fold inside the update
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -q --timeout 200 --timeout-method thread"
B="python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 200 --warmup 20"
tools/gpu_steps.sh \
 "400 r5w/tests.log $T tests/test_gpu_train.py tests/test_gpu_autograph.py tests/test_gpu_parity.py -k 'adam or trajectory or clip or train or graph'" \
 "300 r5w/c2.log $B" \
 "300 r5w/c5.log $B --config c5"
