# wave/lane crossover after lane kernel v4 (kernel us), box rows, cold
mkdir -p gpurun_out
b() { f=gpurun_out/x_$(echo "$@" | tr ' -=' '___').json
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 10 --warmup 2 "$@" > $f 2>gpurun_out/x_err.log || { cat gpurun_out/x_err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(' '.join(sys.argv[2:]), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:12])" $f "$@"; }
for B in 1024 2048 4096 8192; do for be in wave lane; do b --config c2 --batch $B --backend $be; done; done
for B in 1024 2048 4096 6144; do for be in wave lane; do b --config c2 --horizon 30 --batch $B --backend $be; done; done
for B in 256 512 1024; do for be in wave lane; do b --config c4 --batch $B --backend $be --grouped off; done; done
for B in 1920 4096 8192 16384; do b --config c4 --horizon 20 --batch $B --backend wave --grouped on; b --config c4 --horizon 20 --batch $B --backend lane; done
for B in 480 960 1920; do b --config c4 --batch $B --backend wave --grouped on; done
for be in wave lane; do b --config c5_cold --backend $be; b --config c5 --backend $be; done
