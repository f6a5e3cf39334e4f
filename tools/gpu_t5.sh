mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt5.log 2>&1; rc=$?
tail -2 gpurun_out/pt5.log
grep -qE "illegal memory|Memory access fault|HSA_STATUS_ERROR" gpurun_out/pt5.log && exit 99
[ $rc -ne 0 ] && exit $rc
for t in 512 1024 2048; do
timeout -k 10 200 python tools/tune_variants.py run --tile $t > gpurun_out/tune5_$t.log 2>&1 || exit $?
echo "tile $t"; grep -o '"spass_us": [0-9.]*, "cpass_us": [0-9.]*, "cfinish_us": [0-9.]*\|"variant": "[a-z0-9]*"' gpurun_out/tune5_$t.log | paste - - 
done
