TAG=r04e STEPS="fused rvqb stamps" bash tools/gpu/r04.sh && timeout -k 10 120 python tools/rvq_chain_stamps.py > gpurun_out/r04e_chain_stamps.log 2>&1; tail -30 gpurun_out/r04e_chain_stamps.log
