"""blendtorch for MI355X: stream Blender (or headless) renderings into PyTorch.

Sub-packages
------------
btt        PyTorch-side API (datasets, launcher, duplex, remote envs, GPU loader)
btb        Blender-side API (publisher, animation, renderer, camera, envs)
transport  pyzmq-compatible native ZMTP transport
ops        hand-written gfx950 HIP kernels (decode, color transform, projection)
parallel   RCCL/xGMI sharding of batches across the GPUs of a node
models     consumer models used by examples and the benchmark
utils      config, metrics, tracing helpers
"""
__version__ = '0.2.0'
