# dword-aligned XXH3 loads: A/B against the previous build (mb_lib_kv1.so)
set -e
mkdir -p gpurun_out
o=gpurun_out/alab.log
: > $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/al_pytest.log 2>&1 || { tail -40 gpurun_out/al_pytest.log; exit 1; }
tail -2 gpurun_out/al_pytest.log >> $o
A="microbench/mb_lib_kv1.so microbench/mb_lib_al1.so"
echo "== xxh3 mix" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --mixed --blocks 262144 >> $o 2>&1
echo "== xxh3 4K aligned" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 >> $o 2>&1
echo "== xxh3 4097 stride" >> $o; timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --block 4097 --blocks 262144 >> $o 2>&1
echo "== xxh3 wave 4097 stride" >> $o; MCK_XXH3_DRIVER=wave timeout -k 10 120 python microbench/ab.py $A --kind xxh3 --block 4097 --blocks 262144 >> $o 2>&1
echo "== bench sst" >> $o; timeout -k 10 180 python bench.py --workload sst >> $o 2>&1
echo "== bench kv" >> $o; timeout -k 10 180 python bench.py --workload kv >> $o 2>&1
echo "== bench xxh3" >> $o; timeout -k 10 180 python bench.py --workload xxh3 >> $o 2>&1
cat $o
