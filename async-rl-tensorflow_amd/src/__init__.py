"""MI355X-native drop-in for the rollout + gradient path of datavizweb/async-rl-tensorflow.

Module names mirror the reference's ``src/`` package (agent, network, environment, history,
ops, base, utils) so ``from src.agent import Agent`` keeps working; the arithmetic runs in
hand-written HIP kernels (``../csrc``) behind the C-ABI of ``include/a3c_hip.h``.
"""
