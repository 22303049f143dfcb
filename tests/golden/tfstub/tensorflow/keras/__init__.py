"""Stub `tensorflow.keras` (test infrastructure only): base classes so reference modules import."""
from . import layers  # noqa: F401


class Model(object):
    def __init__(self, *args, **kwargs):
        pass


class _Applications(object):
    def __getattr__(self, name):
        raise RuntimeError("keras.applications.%s is not available in the golden stub" % name)


applications = _Applications()
