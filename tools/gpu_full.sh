set -o pipefail
tools/gpu_steps.sh "?900 full/tests.log python3 -m pytest tests -m gpu -x -q" "600 full/bench.log python3 bench.py --no-cpu-baseline"
