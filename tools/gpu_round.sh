# GPU sweep used during development: full GPU suite + back-end crossover by batch size
mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t_gpu8.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu8.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 200 python bench.py --no-cpu --config $1 --backend $2 --batch $3 --steps 30 > gpurun_out/x_$1_$2_$3.json 2>gpurun_out/x_$1_$2_$3.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/x_$1_$2_$3.json'));print('$1 $2 B=$3', '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3))"; }
for B in 256 1024 1536 2048 3072 4096 8192; do run c2 wave $B; run c2 lane $B; done
for B in 1024 2048 4096; do run c4 wave $B; run c4 lane $B; done
