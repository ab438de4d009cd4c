mkdir -p gpurun_out/r6h
for i in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r6h/b$i.json 2> gpurun_out/r6h/b$i.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r6h/b$i.json').read().strip().splitlines()[-1]); print($i, d['ms_per_step'], d['kernel_ms_p10_p50_p90'], d['warmup_effective'], d['warmup_settle_ms_per_step'])"
done
