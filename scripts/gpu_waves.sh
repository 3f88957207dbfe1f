python build.py > gpurun_out/build.log 2>&1 || exit 1
for w in 4 8; do
timeout -k 10 200 python tools/stamp_qstep.py --chunk 64 --waves $w --out gpurun_out/stamps_w$w.md > gpurun_out/stamps_w$w.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --chunk 64 --step-waves $w > gpurun_out/bench_w$w.log 2>&1 || exit 1
done
