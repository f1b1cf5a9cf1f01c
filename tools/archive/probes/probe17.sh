V=async-rl-tensorflow_amd/lib/var
for args in "--envs 512" "--frames84" "--lstm --game SpaceInvaders-v0" "--game Breakout-v0"; do
echo "### $args"
AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_LIB=$V/lxall/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids || exit 1
done
