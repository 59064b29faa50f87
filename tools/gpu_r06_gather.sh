#!/bin/bash
# Random-record gather ceiling (tools/microbench/gather_ceiling.hip): the sweep, then two PMC passes
# (fabric requests by size) over the 400 MB / 5-waves cases, each GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 tools/microbench/gather_ceiling > $O/gather_ceiling.jsonl 2> $O/gather_ceiling.err && echo "sweep ok" &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- tools/microbench/gather_ceiling 400,4096 5 > $O/pmc_fetch.log 2>&1 && echo "fetch ok" &&
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_REQ_sum --kernel-trace -d $O/pmc_tcc -o run --output-format csv -- tools/microbench/gather_ceiling 400,4096 5 > $O/pmc_tcc.log 2>&1 && echo "tcc ok"
