"""Stub (test infrastructure only)."""


class Classifiers(object):
    @staticmethod
    def get(name):
        raise RuntimeError("classification_models is not available in the golden stub")
