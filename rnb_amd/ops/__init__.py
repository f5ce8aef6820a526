"""Hot ops: HIP/CDNA4 kernels (librnb_kernels.so) with torch numerics mirrors.

* ``conv.ConvLayer``   implicit-GEMM NDHWC bf16 conv + fused bias/residual/ReLU
* ``video``            synthetic decode, preprocess, pooled head, per-video reduce
* ``native``           ctypes bindings + loader for the in-tree .so files
"""
