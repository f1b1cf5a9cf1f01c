"""CPU oracle for the rollout + gradient path (TEST INFRASTRUCTURE ONLY).

This package is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``async-rl-tensorflow_amd/``) must never route through it.

Modules
-------
ref_cpu        numpy restatement of the reference's arithmetic, each function citing
               the reference file:line it follows (environment.py, history.py,
               agent.py, network.py, ops.py, main.py).
philox         Philox4x32-10 counter RNG (build-defined; replayed bit-exactly on GPU).
synthetic_env  build-defined stand-in for gym/ALE (absent from the image), with the
               reference's act/new_game/new_random_game semantics.

Pinning: preprocessing and history are pinned by golden vectors produced by the
reference's own ``src/environment.py`` / ``src/history.py`` (tests/golden/); the
network/loss/optimizer arithmetic is **parity unpinned** against a reference
execution (TensorFlow 0.x is absent and unpinned) and is cross-checked instead
against torch CPU autograd as an independent implementation.
"""
