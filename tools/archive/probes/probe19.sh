AB_MODES=overlap AB_REPS=2 timeout -k 10 800 bash tools/ab.sh "A3C_X=0" "A3C_RB_EVENT=1" "A3C_CB_LEAN=1" "A3C_CB_LEAN=1 A3C_RB_EVENT=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=2 AB_ARGS="--frames84" timeout -k 10 600 bash tools/ab.sh "A3C_X=0" "A3C_RB_EVENT=1" 2>&1 | grep -v amdgpu.ids
