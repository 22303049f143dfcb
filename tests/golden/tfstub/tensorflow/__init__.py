"""Numpy-backed stand-in for the handful of TensorFlow-2 eager *elementwise* ops that the
reference's target-assignment / loss / anchor functions call.

TEST INFRASTRUCTURE ONLY.  It exists so that `tests/golden/make_golden.py` can execute the
reference's own numpy-level code (`FCOS/fcos.py:format_data/model_loss`,
`RetinaNet/retinanet_module.py:RetinaNet.format_data`, `CenterNet/*format_data`, ...) in this
container, where TensorFlow is not installed, and record their outputs as golden vectors.
It implements no detector algorithm; every op here is a 1-line numpy equivalent.

TF2 semantics reproduced (they decide the bits of the golden vectors):
* a Tensor keeps its dtype; python scalars and numpy arrays entering a binary op with a
  Tensor are converted to the Tensor's dtype (TF `binary_op_wrapper` / `args_to_matching_eager`),
  so `float64_ndarray - fp32_tensor` is computed in fp32, as in TF;
* `tensor.numpy()` returns a copy (TF2 `EagerTensor.numpy`);
* `__array_priority__ = 100` so numpy scalars/arrays defer to the Tensor's reflected ops,
  while `np.maximum(0, tensor)` etc. still work through `__array__`;
* python floats become float32 tensors (TF default).
"""
import numpy as _np

float32 = _np.float32
float64 = _np.float64
int32 = _np.int32
int64 = _np.int64
bool = _np.bool_


def _default_dtype(v):
    if isinstance(v, (_np.generic, _np.ndarray)):
        return None                      # numpy values keep their dtype (np.float64 is a float!)
    if isinstance(v, (_np.bool_,)) or v is True or v is False:
        return _np.bool_
    if isinstance(v, int):
        return _np.int32
    if isinstance(v, float):
        return _np.float32
    return None


class Tensor(object):
    __array_priority__ = 100

    def __init__(self, value, dtype=None):
        if isinstance(value, Tensor):
            value = value._a
        if dtype is None:
            dtype = _default_dtype(value)
            if dtype is None and isinstance(value, (list, tuple)):
                arr = _np.array([x._a if isinstance(x, Tensor) else x for x in value])
                if arr.dtype == _np.float64 and not any(
                        isinstance(x, (_np.ndarray, _np.generic, Tensor)) for x in value):
                    arr = arr.astype(_np.float32)
                elif arr.dtype == _np.int64 and not any(
                        isinstance(x, (_np.ndarray, _np.generic, Tensor)) for x in value):
                    arr = arr.astype(_np.int32)
                self._a = arr
                return
        self._a = _np.array(value, dtype=dtype)

    # --- conversion -------------------------------------------------------------------
    @property
    def dtype(self):
        return self._a.dtype.type

    @property
    def shape(self):
        return tuple(self._a.shape)

    def numpy(self):
        return self._a.copy()

    def __array__(self, dtype=None, copy=None):
        return self._a if dtype is None else self._a.astype(dtype)

    def __len__(self):
        return len(self._a)

    def __int__(self):
        return int(self._a)

    def __float__(self):
        return float(self._a)

    def __index__(self):
        return int(self._a)

    def __bool__(self):
        return bool(self._a)

    def __getitem__(self, idx):
        if isinstance(idx, Tensor):
            idx = idx._a
        return Tensor(self._a[idx])

    def __iter__(self):
        for i in range(len(self._a)):
            yield Tensor(self._a[i])

    def __repr__(self):
        return "StubTensor(%r)" % (self._a,)

    # --- arithmetic: other operand converted to this tensor's dtype --------------------
    def _conv(self, other):
        if isinstance(other, Tensor):
            if other._a.dtype != self._a.dtype:
                raise TypeError("dtype mismatch %s vs %s" % (self._a.dtype, other._a.dtype))
            return other._a
        return _np.asarray(other).astype(self._a.dtype)

    def _bin(self, other, fn, reflect=False):
        o = self._conv(other)
        r = fn(o, self._a) if reflect else fn(self._a, o)
        return Tensor(_np.asarray(r))

    def __add__(self, o): return self._bin(o, _np.add)
    def __radd__(self, o): return self._bin(o, _np.add, True)
    def __sub__(self, o): return self._bin(o, _np.subtract)
    def __rsub__(self, o): return self._bin(o, _np.subtract, True)
    def __mul__(self, o): return self._bin(o, _np.multiply)
    def __rmul__(self, o): return self._bin(o, _np.multiply, True)

    def __truediv__(self, o):
        if _np.issubdtype(self._a.dtype, _np.integer):
            a = self._a.astype(_np.float64)
            return Tensor(a / _np.asarray(o._a if isinstance(o, Tensor) else o, _np.float64))
        return self._bin(o, _np.divide)

    def __rtruediv__(self, o):
        return self._bin(o, _np.divide, True)

    def __neg__(self): return Tensor(-self._a)
    def __abs__(self): return Tensor(_np.abs(self._a))
    def __lt__(self, o): return self._bin(o, _np.less)
    def __le__(self, o): return self._bin(o, _np.less_equal)
    def __gt__(self, o): return self._bin(o, _np.greater)
    def __ge__(self, o): return self._bin(o, _np.greater_equal)
    def __pow__(self, o): return self._bin(o, _np.power)


def _t(x, dtype=None):
    if isinstance(x, Tensor):
        return x if dtype is None else Tensor(x._a.astype(dtype))
    if isinstance(x, _np.ndarray) or isinstance(x, _np.generic):
        return Tensor(_np.asarray(x) if dtype is None else _np.asarray(x).astype(dtype))
    return Tensor(x, dtype)


def _pair(a, b):
    """Convert a binary-op operand pair the way TF's op wrappers do (first tensor's dtype)."""
    if isinstance(a, Tensor):
        return a, Tensor(a._conv(b))
    if isinstance(b, Tensor):
        return Tensor(b._conv(a)), b
    ta = _t(a)
    return ta, Tensor(ta._conv(b))


def constant(value, dtype=None):
    return _t(value, dtype)


def convert_to_tensor(value, dtype=None):
    return _t(value, dtype)


def cast(x, dtype):
    return Tensor(_np.asarray(x._a if isinstance(x, Tensor) else x).astype(dtype))


def _arr(x):
    return x._a if isinstance(x, Tensor) else _np.asarray(x)


def concat(values, axis):
    return Tensor(_np.concatenate([_arr(v) for v in values], axis=axis))


def stack(values, axis=0):
    return Tensor(_np.stack([_arr(v) for v in values], axis=axis))


def expand_dims(x, axis):
    return Tensor(_np.expand_dims(_arr(_t(x)), axis))


def squeeze(x, axis=None):
    return Tensor(_np.squeeze(_arr(x), axis=axis))


def reduce_sum(x, axis=None):
    if isinstance(x, (list, tuple)):
        x = stack(x)
    a = _arr(_t(x))
    axis = tuple(axis) if isinstance(axis, list) else axis
    return Tensor(_np.sum(a, axis=axis).astype(a.dtype))


def reduce_max(x, axis=None):
    a = _arr(_t(x))
    return Tensor(_np.max(a, axis=axis))


def reduce_min(x, axis=None):
    a = _arr(_t(x))
    return Tensor(_np.min(a, axis=axis))


def reduce_mean(x, axis=None):
    a = _arr(_t(x))
    return Tensor(_np.mean(a, axis=axis).astype(a.dtype))


def exp(x): return Tensor(_np.exp(_arr(_t(x))))
def abs(x): return Tensor(_np.abs(_arr(_t(x))))
def square(x): return Tensor(_np.square(_arr(_t(x))))


def multiply(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.multiply(a._a, b._a))


def add(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.add(a._a, b._a))


def subtract(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.subtract(a._a, b._a))


def divide(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.divide(a._a, b._a))


def pow(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.power(a._a, b._a))


def minimum(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.minimum(a._a, b._a))


def maximum(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.maximum(a._a, b._a))


def less(a, b):
    a, b = _pair(a, b)
    return Tensor(_np.less(a._a, b._a))


def where(cond, x, y):
    x, y = _pair(x, y)
    return Tensor(_np.where(_arr(cond), x._a, y._a))


def range(start, limit=None, delta=1, dtype=None):
    if limit is None:
        start, limit = 0, start
    dt = dtype if dtype is not None else (
        _np.float32 if isinstance(start, float) or isinstance(limit, float) else _np.int32)
    return Tensor(_np.arange(_np.asarray(_arr(start)).item(), _np.asarray(_arr(limit)).item(),
                             _np.asarray(_arr(delta)).item(), dtype=dt))


def meshgrid(*args):
    return [Tensor(g) for g in _np.meshgrid(*[_arr(a) for a in args])]


def shape(x):
    return Tensor(_np.array(_arr(x).shape, dtype=_np.int32))


def zeros_like(x):
    return Tensor(_np.zeros_like(_arr(x)))


def ones_like(x):
    return Tensor(_np.ones_like(_arr(x)))


def constant_initializer(value):
    return value


def ensure_shape(x, shape):
    return x


class _Math(object):
    @staticmethod
    def log(x): return Tensor(_np.log(_arr(_t(x))))

    @staticmethod
    def sqrt(x): return Tensor(_np.sqrt(_arr(_t(x))))

    @staticmethod
    def add(a, b): return add(a, b)

    @staticmethod
    def divide_no_nan(a, b):
        a, b = _pair(a, b)
        with _np.errstate(divide="ignore", invalid="ignore"):
            r = _np.where(b._a == 0, 0, a._a / b._a)
        return Tensor(r.astype(a._a.dtype))

    @staticmethod
    def argmax(x, axis=None): return Tensor(_np.argmax(_arr(x), axis=axis))


math = _Math()


class _NN(object):
    @staticmethod
    def sigmoid(x):
        a = _arr(_t(x))
        return Tensor((1.0 / (1.0 + _np.exp(-a))).astype(a.dtype))

    @staticmethod
    def relu(x):
        a = _arr(_t(x))
        return Tensor(_np.maximum(a, 0).astype(a.dtype))

    @staticmethod
    def sigmoid_cross_entropy_with_logits(labels=None, logits=None):
        # TF's stable form: max(x, 0) - x * z + log(1 + exp(-|x|)), in the logits' dtype
        x = _arr(_t(logits))
        z = _arr(_t(labels)).astype(x.dtype)
        return Tensor((_np.maximum(x, 0) - x * z + _np.log1p(_np.exp(-_np.abs(x)))).astype(x.dtype))


nn = _NN()


class Variable(Tensor):
    def __init__(self, initial_value=0.0, trainable=True, name=None, **kw):
        Tensor.__init__(self, initial_value)


from . import keras  # noqa: E402,F401
