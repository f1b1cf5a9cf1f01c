set -o pipefail
echo "### M2: conv backward workgroups (with the solo LDS reservation)"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_CB_NWG=214" "A3C_CB_NWG=256" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M1"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_CB_NWG=214" "A3C_CB_NWG=256" 2>&1 | grep -v amdgpu.ids || exit 1
