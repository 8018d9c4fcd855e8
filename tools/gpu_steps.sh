#!/bin/bash
# Run GPU steps in order, each under its own time limit. Any non-zero status ends the chain, so
# nothing more touches the GPU after a fault, abort or timeout — except a step prefixed with "?",
# whose plain failure (exit 1, e.g. a failed pytest assertion) is tolerated; pytest reports a
# device fault as a crash (not 1) or in its log, which the step after it never masks.
# usage: tools/gpu_steps.sh "<timeout_s> <log> <cmd...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  soft=0
  if [ "${spec:0:1}" = "?" ]; then soft=1; spec="${spec:1}"; fi
  read -r t log cmd <<<"$spec"
  mkdir -p "$(dirname "gpurun_out/$log")"
  echo "[gpu_steps] $(date +%T) start: $cmd (limit ${t}s) -> $log"
  timeout -k 10 "$t" bash -c "$cmd" >"gpurun_out/$log" 2>&1
  rc=$?
  echo "[gpu_steps] $(date +%T) rc=$rc: $cmd"
  grep -v amdgpu "gpurun_out/$log" | tail -n 6 | cut -c1-600
  if [ $rc -ne 0 ]; then
    if [ $soft -eq 1 ] && [ $rc -eq 1 ] && ! grep -qi "illegal memory\|memory access fault\|hipErrorIllegal\|core dumped" "gpurun_out/$log"; then
      continue
    fi
    echo "[gpu_steps] stopping after rc=$rc"
    exit $rc
  fi
done
