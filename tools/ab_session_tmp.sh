mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_full_size.py -m gpu -x -v --timeout 120 --timeout-method thread -k "r6" > gpurun_out/gputests_r6len.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/gputests_r6len.log)"
grep -E "PASS|FAIL" gpurun_out/gputests_r6len.log | head -20
