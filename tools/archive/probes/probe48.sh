set -o pipefail
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/b48.json 2> gpurun_out/b48.err && python3 -c "import json;d=json.load(open('gpurun_out/b48.json'));print('M1', d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['kernels']['k_fc_part'])"
timeout -k 10 300 python3 bench.py --frames84 --no-cpu-baseline > gpurun_out/b48m2.json 2> gpurun_out/b48m2.err && python3 -c "import json;d=json.load(open('gpurun_out/b48m2.json'));print('M2', d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
