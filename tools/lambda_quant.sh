cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in 24576 36864 49152 50000 51200; do
  timeout -k 10 200 python -u bench.py --cols $c --steps 20 --warmup 5 --no-cpu-baseline --no-fitted > gpurun_out/lq_$c.json 2> gpurun_out/lq_$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lq_$c.json'));r=d['roofline'];print($c, round(d['value'],1), r['kernel'], round(r['kernel_ms_avg']*1e3,1), d.get('phases_ms'))"
done
