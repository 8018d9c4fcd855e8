#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r3_hop.sh && bash tools/gpu_r3_stamps.sh
