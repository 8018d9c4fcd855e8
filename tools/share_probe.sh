#!/bin/bash
# Two independent single-rank graph-mode benches on ONE GPU at the same time (no collective):
# separates a GPU-sharing artefact from the multi-rank code path.
python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > gpurun_out/share/a.log 2>&1 &
pa=$!
python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > gpurun_out/share/b.log 2>&1 &
pb=$!
wait $pa; ra=$?
wait $pb; rb=$?
echo "rc $ra $rb"
exit $(( ra | rb ))
