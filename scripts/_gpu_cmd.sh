V=scripts/variants
bash scripts/gpu_evidence.sh c2 32 512 768 x6 && mkdir -p gpurun_out/ab \
&& bash scripts/gpu_ab.sh scripts/kbench_x6.py "x6 down" base $V/libnofill.so $V/libpf2.so $V/libpf2e.so > gpurun_out/ab/down_fill.log 2>&1 && echo "ab ok"
