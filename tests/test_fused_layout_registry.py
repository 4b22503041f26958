"""The fused PS worker's TF-layout mapping comes from the variable registry (get_vars,
utils.py:3-8; pairing by position, worker.py:76-77), not from hard-coded names: renaming the
outer scope keeps the conversion round-tripping."""
import pytest
import torch

from distributedtensorflowexample_amd import variables as vs
from distributedtensorflowexample_amd.models.dense import make_ps_model
from distributedtensorflowexample_amd.ops import mlp_step
from distributedtensorflowexample_amd.train.worker import (REFERENCE_MLP_NAMES,
                                                           build_worker_variables,
                                                           flat_to_tf_vars, fused_tf_names,
                                                           split_tf_flat, tf_vars_to_flat)


@pytest.mark.parametrize("scope", ["global", "ps_vars", "tower0/global"])
def test_fused_names_follow_registry_scope(scope):
    reg = vs.VariableRegistry()
    gvars, trainable = build_worker_variables(make_ps_model("mlp", "", None), reg, scope)
    names = fused_tf_names(trainable)
    assert all(n.startswith(scope + "/") for n in names)
    assert [n[len(scope) + 1:] for n in names] == [n[len("global/"):] for n in REFERENCE_MLP_NAMES]
    assert any(v.name == scope + "/global_step" for v in gvars)
    g = torch.Generator().manual_seed(0)
    p = torch.randn(mlp_step.NPARAM, generator=g)
    tf = flat_to_tf_vars(p, names)
    assert set(tf) == set(names)
    back = tf_vars_to_flat(tf, torch.zeros_like(p), names)
    assert torch.equal(back, p)
    # the TF-layout flat (what to_tf_layout writes / the ps pull buffer holds) splits into the
    # same tensors, in the registry's order
    flat = torch.cat([tf[n].contiguous().reshape(-1) for n in names])
    views = split_tf_flat(flat, names)
    for n in names:
        assert torch.equal(views[n], tf[n])


def test_fused_names_reject_other_models():
    reg = vs.VariableRegistry()
    _, trainable = build_worker_variables(make_ps_model("mlp", "256,128", "relu"), reg)
    with pytest.raises(ValueError):
        fused_tf_names(trainable)
