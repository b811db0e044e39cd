mkdir -p gpurun_out/ab
bash scripts/gpu_evidence.sh c2 32 512 768 x6 && echo c2 ok \
&& timeout -k 10 900 python bench.py --config 3 > gpurun_out/ab/c3_bench.log 2>&1 && echo c3 ok
