"""Stub `tensorflow.keras.layers` (test infrastructure only). Model-building layers are not
available: golden generation only calls the reference's numpy-level functions."""


class Layer(object):
    def __init__(self, *args, **kwargs):
        pass


def __getattr__(name):
    raise RuntimeError("keras.layers.%s is not available in the golden stub" % name)
