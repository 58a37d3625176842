"""GPU: the bench's whole train-step forward + backward at full BASELINE size against the fp64
oracle (the reference orchestration Models/BuckGNN.py:67-74,323,430-471 over the PyG
restatement), on the exact code path bench.py times, for every SAGE variant of the layer loop:
GraphSage_addAggr (:430-444), GraphSage_meanAggr (:445-458), GraphSage_maxAggr (:459-471) and
GraphSage_addAggr_Shared (:338-352, TRAIN_FINAL.py's default) at h=512 L=6, on a full cfg2 batch
(16 x 71x71 meshes with virtual edges: N = 80,656, E = 715,872) and a full cfg3 batch (16 meshes
with super nodes of in-degree 5,041: N = 80,672, E = 792,992); folded node encoder + bgnn_mlp2
head (sum / mean) or the unfolded encoder (max), fused layers, BatchNorm in train mode, dropout 0
(torch's dropout RNG cannot be matched). Checked: the 16 predictions and the RelativeErrorLoss
within the north star's 1e-4, every used parameter's gradient checksum, the whole gradient
tensors within 1e-3 relative L2 per parameter (with a noise floor for the gradients that are
exactly 0 in exact arithmetic), BatchNorm running statistics, and the set of parameters with
gradients.

Max aggregation (aggr='max'): the gradient of each (target, channel) goes to ONE argmax source,
so an f32 forward that orders two near-equal neighbours differently from fp64 routes that
element's gradient elsewhere. The test makes this explicit instead of widening a tolerance: it
captures every layer's GPU argmax and its layer input, checks that each place where the GPU's
choice differs from fp64's first argmax is a near tie -- fp64 margin max - x_choice at most twice
the layer input's largest f32 error (measured, max |x_gpu - x_fp64|) -- and then evaluates the
fp64 backward along the GPU's choices, so the whole-tensor gradient bounds are the same as for
the linear aggregations. The flip counts are printed.

Every layer's normalised SAGEConv output (the north star's "match the reference CPU SAGEConv outputs
on identical edge_index/x within 1e-4 fp32", Models/BuckGNN.py:434) is checked twice at full size:
(1) literally -- the fp64 oracle's SAGEConv (oracle/pyg_ref.py) evaluated on the GPU layer's own
input x (for the folded first layer, x = h W_in^T + b_in from the GPU's encoder hidden h, in fp64)
against the GPU's output, max |diff| <= 1e-4; (2) along the whole chain -- the fp64 oracle's
layer-i output against the GPU's, max |diff| <= 1e-4 (every earlier layer's rounding included)."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn import buckgnn, fused
from bgnn import synthetic as S
from oracle import buckgnn_ref as R
from oracle import pyg_ref
from recipe import grad_checksum

pytestmark = pytest.mark.gpu

VARIANTS = ["GraphSage_addAggr", "GraphSage_meanAggr", "GraphSage_maxAggr", "GraphSage_addAggr_Shared"]


class _ForcedMax(torch.autograd.Function):
    """fp64 segment max whose backward follows a given argmax (the GPU's), after checking that
    every disagreement with fp64's own first argmax is a near tie (margin <= tol)."""

    @staticmethod
    def forward(ctx, src, index, dim_size, eid, tol, stats):
        idx = index.view(-1, 1).expand_as(src)
        out = src.new_zeros((dim_size, src.size(1))).scatter_reduce_(0, idx, src, reduce="amax", include_self=False)
        n = src.size(0)
        pos = torch.arange(n).view(-1, 1).expand_as(src)
        hit = src == out.index_select(0, index)
        first = torch.full(out.shape, n, dtype=torch.long)
        first.scatter_reduce_(0, idx, torch.where(hit, pos, torch.full_like(pos, n)), reduce="amin", include_self=True)
        del hit, pos
        valid = first < n
        assert torch.equal(eid < n, valid), "GPU argmax on an empty row or none on a non-empty one"
        flip = valid & (eid != first)
        if flip.any():
            rows, cols = torch.nonzero(flip, as_tuple=True)
            margin = out[rows, cols] - src[eid[rows, cols], cols]
            assert bool((index[eid[rows, cols]] == rows).all()), "GPU argmax outside the row's edges"
            stats.append((int(flip.sum()), float(margin.max()), tol))
            assert float(margin.max()) <= tol, ("argmax flip beyond a near tie", float(margin.max()), tol)
        else:
            stats.append((0, 0.0, tol))
        ctx.save_for_backward(torch.where(valid, eid, torch.full_like(eid, n)))
        ctx.n = n
        return out

    @staticmethod
    def backward(ctx, g):
        (sel,) = ctx.saved_tensors
        n = ctx.n
        gs = g.new_zeros((n + 1, g.size(1)))
        gs.scatter_(0, sel, g)
        return gs[:n], None, None, None, None, None


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
@pytest.mark.parametrize("model_name", VARIANTS)
def test_full_size_train_step_matches_fp64_oracle(dev, monkeypatch, cfg, model_name):
    b = S.make_config_batch(cfg)
    assert (b.num_nodes, b.num_edges) == {"cfg2": (80656, 715872), "cfg3": (80672, 792992)}[cfg]
    is_max = model_name == "GraphSage_maxAggr"
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=model_name)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    folds = []
    real_layer = buckgnn.sage_layer
    monkeypatch.setattr(buckgnn, "sage_layer", lambda *a, **k: folds.append(k.get("w_in") is not None)
                        or real_layer(*a, **k))
    layer_io = []   # per layer: (SAGEConv input as the GPU layer received it, normalised output o)
    real_glue = fused._glue_fwd

    def glue_spy(o, bn_part, slots, x_prev, *a, **k):
        layer_io.append((x_prev.detach().cpu(), o.detach().cpu()))
        return real_glue(o, bn_part, slots, x_prev, *a, **k)
    monkeypatch.setattr(fused, "_glue_fwd", glue_spy)
    captured = []   # max: per layer (input x [N, C] f32, argmax [N, C] as forward-CSR positions)
    if is_max:
        real_mt = fused._max_transform

        from bgnn import ops

        def spy(x, w_l, w_r, graph, *a, **k):
            y, agg, arg = real_mt(x, w_l, w_r, graph, *a, **k)
            pos = ops.max_arg_positions(graph.fwd, arg, x.size(0), x.size(1))   # CSR positions, -1: empty row
            captured.append((x.detach().cpu(), pos.cpu()))
            return y, agg, arg
        monkeypatch.setattr(fused, "_max_transform", spy)
    bd = b.to(dev)
    pred, _ = m(bd.x, bd.edge_index, bd.edge_attr, bd.batch)
    loss = bgnn.RelativeErrorLoss()(pred, bd.y)
    loss.backward()
    torch.cuda.synchronize()
    # the bench's path: the encoder folded into the first layer for sum / mean, not for max
    assert folds == ([False] * 6 if is_max else [True] + [False] * 5)
    assert len(captured) == (6 if is_max else 0)
    got = {k: p.grad.detach().cpu().double().numpy() for k, p in m.named_parameters() if p.grad is not None}
    state = {k: v.detach().cpu() for k, v in m.state_dict().items() if "running_" in k}
    pred_g, loss_g = pred.detach().cpu().double(), float(loss.item())
    del m, bd, pred, loss
    torch.cuda.empty_cache()

    # fp64 oracle on the host (~25-60 s with 8-16 threads)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    assert len(layer_io) == 6
    attr, aggr, _ = R.SAGE[model_name]
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    gpu_o = [o for _, o in layer_io]
    worst_in = []
    for i, (x_in, o) in enumerate(layer_io):   # (1) identical input x, fp64 SAGEConv, literal 1e-4
        pre = attr if model_name.endswith("_Shared") else f"{attr}.{i}"
        x_in = x_in.double()
        if i == 0 and folds and folds[0]:   # the folded layer received the encoder hidden h
            last = max(int(k.split(".")[1]) for k in sd64 if k.startswith("node_encoder."))
            x_in = torch.nn.functional.linear(x_in, sd64[f"node_encoder.{last}.weight"],
                                              sd64[f"node_encoder.{last}.bias"])
        ref_o = R.sage_conv(sd64, pre, x_in, b.edge_index, aggr)
        d = float((o.double() - ref_o).abs().max())
        worst_in.append(d)
        assert d <= 1e-4, ("SAGEConv output vs fp64 on the identical input", i, d)
    del layer_io
    print("per-layer SAGEConv max |GPU - fp64| on the identical input:", [f"{d:.2e}" for d in worst_in])
    chain_o = []
    real_conv = R.sage_conv
    monkeypatch.setattr(R, "sage_conv", lambda *a, **k: chain_o.append(real_conv(*a, **k)) or chain_o[-1])
    flips = []
    if is_max:
        # forward-CSR position -> edge id (the CSR is a stable sort of edge_index by target)
        perm = torch.from_numpy(np.argsort(b.edge_index[1].numpy(), kind="stable"))
        E = b.edge_index.size(1)
        layer = [0]
        real_agg = pyg_ref.sage_aggregate

        def forced_aggregate(x, edge_index, aggr):
            assert aggr == "max"
            k = layer[0]
            layer[0] += 1
            xg, arg = captured[k]
            # the layer input's largest f32 error: the flip allowance is twice it
            tol = 2.0 * float((xg.double() - x.detach()).abs().max())
            arg = arg.long()
            eid = torch.where(arg >= 0, perm[arg.clamp_min(0)], torch.full_like(arg, E))
            msg = x.index_select(0, edge_index[0])
            return _ForcedMax.apply(msg, edge_index[1], x.size(0), eid, tol, flips)
        monkeypatch.setattr(pyg_ref, "sage_aggregate", forced_aggregate)
        monkeypatch.setattr(R, "sage_aggregate", forced_aggregate, raising=False)
    st = {k: v.double().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd.items()}
    pred_o = R.forward(st, model_name, b.x.double(), b.edge_index, b.batch, True, "mean", 0.0)
    loss_o = R.relative_error_loss(pred_o, b.y.double())
    loss_o.backward()
    if is_max:
        assert len(flips) == 6
        print("argmax flips per layer (count, largest fp64 margin, allowance):", flips)

    assert len(chain_o) == 6
    worst_chain = [float((o.double() - c.detach()).abs().max()) for o, c in zip(gpu_o, chain_o)]
    print("per-layer SAGEConv max |GPU - fp64| along the chain:", [f"{d:.2e}" for d in worst_chain])
    assert max(worst_chain) <= 1e-4, worst_chain
    del gpu_o, chain_o
    np.testing.assert_allclose(pred_g.numpy(), pred_o.detach().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(loss_g, float(loss_o), rtol=1e-4, atol=1e-4)
    ref = {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_allclose(grad_checksum(got[k]), grad_checksum(ref[k]), rtol=2e-3, atol=2e-4, err_msg=k)
    # whole gradient tensors, elementwise in aggregate: per parameter the L2 distance to fp64 within
    # 1e-3 of the parameter's own gradient norm, plus a floor of 1e-5 of the largest per-element RMS
    # gradient of the model (biases feeding a BatchNorm have an exact gradient of 0; their float
    # gradients are rounding noise that a purely relative bound cannot judge)
    rms = max(np.sqrt(np.mean(r ** 2)) for r in ref.values())
    worst = []
    for k in ref:
        err = float(np.linalg.norm(got[k] - ref[k]))
        nrm = float(np.linalg.norm(ref[k]))
        bound = 1e-3 * nrm + 1e-5 * rms * np.sqrt(ref[k].size)
        worst.append((err / max(bound, 1e-300), k, err, nrm))
        assert err <= bound, (k, err, nrm, bound)
    print("largest gradient error / bound:", max(worst)[:2])
    for k, v in state.items():   # running statistics after one train-mode step (momentum 0.1)
        np.testing.assert_allclose(v.numpy(), st[k].detach().numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
