# wave kernel per-launch time vs batch (waves per CU) at N = 20
for B in 64 128 256 512 1024 2048; do
timeout -k 10 100 python bench.py --no-cpu --no-latency --config c2 --batch $B --backend wave --steps 20 > /tmp/w.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('/tmp/w.json'));print($B, 'k %.2f us'%(d['roofline']['kernel_ms_per_launch']*1e3))"
done
