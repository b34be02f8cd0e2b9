# wave/lane crossover after the heading-frame / branch-free / fp64-reference lane kernel (kernel us)
mkdir -p gpurun_out
b() { f=gpurun_out/x2_$(echo "$@" | tr ' -=' '___').json
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 10 --warmup 2 "$@" > $f 2>gpurun_out/x2_err.log || { cat gpurun_out/x2_err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(' '.join(sys.argv[2:]), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:12])" $f "$@"; }
for B in 2048 3072 4096; do for be in wave lane; do b --config c2 --batch $B --backend $be; done; done
for B in 2048 3072 4096; do for be in wave lane; do b --config c2 --horizon 30 --batch $B --backend $be; done; done
for B in 512 768 1024; do for be in wave lane; do b --config c4 --batch $B --backend $be --grouped off; done; done
for be in wave lane; do b --config c5_cold --backend $be; done
