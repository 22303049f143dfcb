"""Stub (test infrastructure only) so RetinaNet/retinanet_module.py imports; never called."""
