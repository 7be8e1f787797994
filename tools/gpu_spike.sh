set -x
cd /root/repo
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python tools/spike_ext.py > gpurun_out/spike.txt 2>&1 && \
timeout -k 10 300 python tools/torch_baseline.py --bs 1200 --dtype bf16 --steps 10 > gpurun_out/base_bf16.txt 2>&1 && \
timeout -k 10 300 python tools/torch_baseline.py --bs 1200 --dtype fp16 --steps 10 > gpurun_out/base_fp16.txt 2>&1 && \
timeout -k 10 300 python tools/torch_baseline.py --bs 400 --dtype fp32 --steps 5 --cl 0 > gpurun_out/base_fp32.txt 2>&1
cat gpurun_out/*.txt
