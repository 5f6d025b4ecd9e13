# generic CRC driver on uniform spans (explicit offsets/lengths) vs the uniform path
set -e
L=speedb_amd/libspeedb_amd.so
for b in 4096 16384 65536; do
  n=$(( (1 << 32) / b ))
  echo "== generic $b"; timeout -k 10 120 python microbench/ab.py $L --kind crc32c --block $b --blocks $n --ragged --rounds 11
  echo "== uniform $b"; timeout -k 10 120 python microbench/ab.py $L --kind crc32c --block $b --blocks $n --rounds 11
  echo "== uniform chunk-layout $b"; MCK_CRC_LAYOUT=0 timeout -k 10 120 python microbench/ab.py $L --kind crc32c --block $b --blocks $n --rounds 11
done
