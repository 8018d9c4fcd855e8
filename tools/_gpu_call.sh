#!/bin/bash
# round-5 working call (overwritten per call): c4 HDF5 stream line (1 M-molecule file), c2 native feed line
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_steps.sh \
 "600 r5s/c4_stream.log python3 bench.py --config c4 --feed stream --stream-mols 1000000 --steps 400 --warmup 20 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r5s/c2_native.log python3 bench.py --feed native --steps 200 --warmup 20 --no-cpu-baseline --no-roofline --no-eager"
