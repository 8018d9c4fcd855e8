set -o pipefail
mkdir -p gpurun_out/lf
timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/lf/a.log 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/lf/b.log 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/lf/c.log 2>&1 && \
AMD_SERIALIZE_KERNEL=0 HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/lf/d.log 2>&1
