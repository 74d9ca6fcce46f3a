"""Drop-in surface checks that need no GPU: the reference's state_dict keys and shapes
load with strict=True into the MI355X modules (HAN, GraphSAGE_Pytorch), and the
reference's error behaviour is kept."""
import numpy as np
import pytest
import torch


def _sd(d, prefix="sd_"):
    return {k[len(prefix):]: torch.from_numpy(np.asarray(d[k])) for k in d if k.startswith(prefix)}


def test_han_state_dict_loads_strict(golden):
    from graphneuralnetwork_amd.han import HANModel
    d = golden("han")
    N, M, Fin, hid, C = (int(v) for v in d["dims"])
    net = HANModel(M, Fin, hid, C, [int(h) for h in d["heads"]], dropout=0.6)
    net.load_state_dict(_sd(d), strict=True)


def test_graphsage_pytorch_state_dicts_load_strict(golden):
    from graphneuralnetwork_amd.graphsage_pytorch import GraphSage, NeighborAggregator, SageGCN
    d = golden("sagepy")
    Fin, B, h0, h1, k0, k1 = (int(v) for v in d["dims"])
    GraphSage(Fin, [h0, h1], [k0, k1]).load_state_dict(_sd(d), strict=True)
    SageGCN(Fin, 12, aggr_neighbor_method="sum", aggr_hidden_method="concat").load_state_dict(
        _sd(d, "sumcat_sd_"), strict=True)
    NeighborAggregator(Fin, 7, use_bias=True).load_state_dict(_sd(d, "biasmean_sd_"), strict=True)


def test_graphsage_pytorch_max_fails_like_the_reference(golden):
    """'max' hands torch.matmul a (values, indices) pair: TypeError, as in the reference."""
    from graphneuralnetwork_amd.graphsage_pytorch import NeighborAggregator
    assert int(golden("sagepy")["max_raises"]) == 1
    with pytest.raises(TypeError):
        NeighborAggregator(8, 3, aggr_method="max")(torch.randn(4, 5, 8))


def test_graphsage_aggregator_rejects_unknown_mode(capsys):
    from graphneuralnetwork_amd.graphsage import Aggregator
    with pytest.raises(RuntimeError):
        Aggregator(torch.randn(2, 3, 4), "SUM")
    assert "请选择合适的聚合函数" in capsys.readouterr().out


def test_sampler_stream_seeds_do_not_collide():
    """Per-(batch seed, layer) RNG keys are hashed: seed + layer would make batch s's
    layer 1 equal batch s+1's layer 0."""
    from graphneuralnetwork_amd.sampler import stream_seed
    keys = {stream_seed(s, layer) for s in range(200) for layer in range(4)}
    assert len(keys) == 800


def test_spmm_accumulate_needs_out():
    """accumulate=True adds into the caller's buffer: without one it is a usage error
    (the check sat after the allocation and never fired)."""
    import torch
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import spmm_forward
    g = CsrGraph(torch.tensor([0, 1]), torch.tensor([0], dtype=torch.int32), torch.ones(1), 1, 1)
    with pytest.raises(ValueError, match="accumulate"):
        spmm_forward(g, torch.ones(1, 4), accumulate=True)
