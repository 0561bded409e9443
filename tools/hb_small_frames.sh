for f in 1 2 4; do timeout -k 10 200 python bench.py --frames $f --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hb_f$f.json 2> gpurun_out/hb_f$f.err || exit 1; done
