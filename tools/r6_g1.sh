cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py::test_lost_retry_cut_is_an_error_not_a_hang tests/test_gpu_parity.py::test_stop_reason_reports_the_engine_cap > gpurun_out/r6_g1_tests.log 2>&1 || { tail -40 gpurun_out/r6_g1_tests.log; exit 1; }
tail -5 gpurun_out/r6_g1_tests.log
bash tools/r6_scan_pmc.sh
