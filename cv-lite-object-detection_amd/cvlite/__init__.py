"""cvlite — MI355X-native training path for the CV-Lite FCOS / CenterNet / RetinaNet detectors.

Host layer over the C ABI in include/cvlite.h (libcvlite_hip.so, gfx950 HIP kernels).  Module
names mirror the reference's model modules: `cvlite.fcos` (FCOS/fcos.py), `cvlite.train_fcos`
(FCOS/train_fcos.py), `cvlite.retinanet` (RetinaNet/retinanet_module.py),
`cvlite.centernet_hourglass` (CenterNet/tf_centernet_hourglass.py), `cvlite.centernet_splat`
(CenterNet/tf_centernet.py).
"""
__version__ = "0.1.0"
