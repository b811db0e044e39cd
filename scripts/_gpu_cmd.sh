mkdir -p gpurun_out/ab
bash scripts/gpu_evidence.sh c5 8 2048 2048 bf16 --config 5 && echo c5 ok
