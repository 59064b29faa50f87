#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/big_mesh_bench.py at 1M triangles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-bigmesh_pmc}; mkdir -p $O
run() { local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$O/$name" -o run --output-format csv -- \
    python3 tools/big_mesh_bench.py --sizes 1000000 --spp 16 > "$O/$name.log" 2>&1; }
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD && echo pmc done
