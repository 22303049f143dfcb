"""Checkpoint round trip of the Keras Adam slots on the host (no GPU): the reference restores
tf.train.Checkpoint(step, model, optimizer) BEFORE training starts (CenterNet/train_hourglass_voc.py:
332-344), i.e. before the optimizer has met its parameters.  cvlite's Adam keeps such restored
slots and applies them when it is bound, instead of silently restarting at m = v = iterations = 0."""
import os
import tempfile

import pytest
import torch

from cvlite import checkpoint as ck
from cvlite.layers import ParamStore, constant
from cvlite.train_centernet import Adam


def _store(n=3):
    st = ParamStore()
    for i in range(n):
        st.add("w%d" % i, (5, 7), constant(0.5 * i))
    st.finalize("cpu", 0)
    return st


def test_adam_slots_restored_before_bind():
    st = _store()
    opt = Adam().bind(st)
    g = torch.Generator().manual_seed(0)
    opt.m.copy_(torch.randn(opt.m.shape, generator=g))
    opt.v.copy_(torch.rand(opt.v.shape, generator=g))
    opt.iterations.fill_(17)
    with tempfile.TemporaryDirectory() as td:
        path = ck.Checkpoint(step=17, optimizer=opt).write(os.path.join(td, "c.pt"))
        fresh = Adam()
        ckpt = ck.Checkpoint(step=0, optimizer=fresh).restore(path)
        assert ckpt.step.value == 17
        assert fresh.m is None and fresh.pending_state is not None   # unbound: kept, not dropped
        fresh.bind(st)
        assert torch.equal(fresh.m, opt.m) and torch.equal(fresh.v, opt.v)
        assert int(fresh.iterations.item()) == 17 and fresh.pending_state is None
        # a bound optimizer takes the slots immediately
        bound = Adam().bind(st)
        ck.Checkpoint(step=0, optimizer=bound).restore(path)
        assert torch.equal(bound.m, opt.m) and int(bound.iterations.item()) == 17


def test_adam_restore_layout_mismatch_raises():
    opt = Adam().bind(_store(3))
    with tempfile.TemporaryDirectory() as td:
        path = ck.Checkpoint(step=1, optimizer=opt).write(os.path.join(td, "c.pt"))
        fresh = Adam()
        ck.Checkpoint(optimizer=fresh).restore(path)
        with pytest.raises(ValueError):
            fresh.bind(_store(4))
