cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export VRVQ_RVQ_WARM=0 VRVQ_STAMPS_NOCHECK=1
for a in "--pt" "--pt --flags 2" "--pt --no-zqis"; do
  echo "### $a"
  timeout -k 10 120 python tools/rvq_fused_stamps.py $a 2>&1 | grep -v amdgpu.ids | grep -E "end|start|done|stored|flags|z_q_is" || exit 1
done
