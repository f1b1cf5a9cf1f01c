set -o pipefail
echo "### M1: rollout stream priority"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_ROLLOUT_PRIO=0" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_ROLLOUT_PRIO=0" 2>&1 | grep -v amdgpu.ids || exit 1
