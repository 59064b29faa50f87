# round 6 session b: checked-build tests, mesh_big tests, counter list, mesh_big bench + PMC
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_checked.py "tests/test_gpu_full_size.py::test_mesh_big_rows" "tests/test_gpu_full_size.py::test_mesh_big_split_items_same_bits" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
tail -15 $O/pytest.log
timeout -k 10 400 python bench.py --config mesh_big --steps 5 --warmup 2 > $O/b_mesh_big.json 2> $O/b_mesh_big.err && echo "mesh_big ok" && head -c 1500 $O/b_mesh_big.json &&
PMC_MEM=1 bash tools/pmc.sh $O/pmc_mesh_big --config mesh_big && echo "pmc ok" &&
cp profiles/pmc_records.json $O/pmc_records.json && python tools/pmc_summary.py $O/pmc_mesh_big mesh4x1000k_1920x1080_64spp_B8 $O/pmc_records.json > $O/pmc_summary.json && echo summary ok
