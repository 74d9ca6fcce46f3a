"""Host logic of the GAT models' hashed dropout (ops.model_dropout / hashed_dropout_ok): where
the HIP kernel does not apply (CPU tensors, p = 0 or 1, eval mode) it is exactly torch's
F.dropout -- after the relabelling gather when one is given. No GPU needed."""
import torch
import torch.nn.functional as F

from graphneuralnetwork_amd import ops


def test_hashed_dropout_ok_conditions():
    x = torch.randn(10, 4)
    assert not ops.hashed_dropout_ok(x, 0.5)  # host tensor
    assert not ops.hashed_dropout_ok(x, 0.0)
    assert not ops.hashed_dropout_ok(x, 1.0)
    assert not ops.hashed_dropout_ok(torch.randn(3, 4, 5), 0.5)


def test_model_dropout_host_is_torch_dropout():
    x = torch.randn(50, 6)
    torch.manual_seed(5)
    a = ops.model_dropout(x, 0.3, True)
    torch.manual_seed(5)
    b = F.dropout(x, 0.3, training=True)
    assert torch.equal(a, b)
    assert ops.model_dropout(x, 0.3, False) is x  # eval: identity, like F.dropout
    assert torch.equal(ops.model_dropout(x, 1.0, True), torch.zeros_like(x))


def test_model_dropout_host_with_permutation():
    x = torch.randn(40, 5, requires_grad=True)
    perm = torch.randperm(40)
    inv = torch.argsort(perm)
    torch.manual_seed(9)
    a = ops.model_dropout(x, 0.4, True, perm, inv)
    torch.manual_seed(9)
    b = F.dropout(x[perm], 0.4, training=True)
    assert torch.equal(a, b)
    a.sum().backward()
    g = x.grad.clone()
    x.grad = None
    b.sum().backward()
    assert torch.equal(g, x.grad)
    # eval: just the relabelling
    assert torch.equal(ops.model_dropout(x, 0.4, False, perm, inv), x[perm])
