# XXH3: bitop3 gathers + realign skipped for dword-aligned spans: parity, A/B
set -e
mkdir -p gpurun_out
o=gpurun_out/x2ab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x2_pytest.log 2>&1 || { tail -40 gpurun_out/x2_pytest.log; exit 1; }
tail -2 gpurun_out/x2_pytest.log >> $o
timeout -k 10 100 python microbench/x3diag.py >> $o 2>&1
MCK_XXH3_DRIVER=wave timeout -k 10 100 python microbench/x3diag.py >> $o 2>&1
A="microbench/mb_lib_x0.so microbench/mb_lib_x2.so"
echo "== mix" >> $o; timeout -k 10 150 python microbench/ab.py $A --kind xxh3 --mixed --blocks 262144 --rounds 15 >> $o 2>&1
echo "== mix align16" >> $o; timeout -k 10 150 python microbench/ab.py $A --kind xxh3 --mixed --align 16 --blocks 262144 --rounds 15 >> $o 2>&1
echo "== wave 4K" >> $o; MCK_XXH3_DRIVER=wave timeout -k 10 150 python microbench/ab.py $A --kind xxh3 --rounds 11 >> $o 2>&1
cat $o
