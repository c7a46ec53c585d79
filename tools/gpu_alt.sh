set -u
mkdir -p gpurun_out
for cfg in "--n 13 --m 4 --batch 1048576" "--n 16 --m 5 --batch 1024 --steps 3 --warmup 1" "--n 10 --m 3 --engine levels" "--n 4 --m 1" "--n 10 --m 1"; do
  name=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python -u bench.py $cfg --no-cpu > gpurun_out/alt_$name.log 2>&1 || { echo "fail $cfg"; exit 1; }
  tail -1 gpurun_out/alt_$name.log
done
bash tools/gpu_session.sh pmc
