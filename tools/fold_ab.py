#!/usr/bin/env python
"""Folded-encoder gradient accuracy against fp64 (tests/test_gpu_fold.py's measure), per
parameter, for the fused path with the weight-by-weight products on torch.mm or on bgnn_gemm,
beside the unfolded path with f16x3 and with f32-MFMA GEMMs (the spread of f32 rounding noise).

    python tools/fold_ab.py [model_name]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "buck-gnn_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from bgnn import fused  # noqa: E402
import test_gpu_fold as T  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "GraphSage_meanAggr"
    dev = torch.device("cuda", 0)
    _, _, _, g_ref = T.run(dev, name, 512, False)
    res = {}
    for flag in (True, False):
        fused.FOLD_WEIGHTS_TORCH = flag
        b, sd, _, g = T.run(dev, name, 512, True)
        res[flag] = g
    # the unfolded path once more with the f32 MFMA GEMMs (same f32 error class, other rounding)
    from bgnn import _lib
    _lib.call("bgnn_set_tuning", 5, 0)
    _, _, _, g_x6 = T.run(dev, name, 512, False)
    _lib.call("bgnn_set_tuning", 5, 2)
    exact = T.oracle_grads(b, sd, name)
    print(f"{'param':45s} {'unfolded':>10s} {'unf/f32mfma':>10s} {'fold/torch':>10s} {'fold/bgnn':>10s}")
    for k in sorted(exact):
        print(f"{k:45s} {T.rel_err(g_ref[k], exact[k]):10.2e} {T.rel_err(g_x6[k], exact[k]):10.2e} "
              f"{T.rel_err(res[True][k], exact[k]):10.2e} {T.rel_err(res[False][k], exact[k]):10.2e}")


if __name__ == "__main__":
    main()


def weight_products(name="GraphSage_addAggr_Shared"):
    """The folded weight-by-weight products on the model's own parameters against fp64."""
    import bgnn
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=name).to(dev)
    blk = m.shared_graphsage_block if name.endswith("Shared") else m.sage_blocks[0]
    wcat = torch.cat([blk.lin_l.weight, blk.lin_r.weight], 0).detach().contiguous()
    w_in, b_in = m.node_encoder[4].weight.detach(), m.node_encoder[4].bias.detach()

    def err(c, r, mag):
        return ((c.double() - r).abs() / mag.clamp_min(1e-300)).max().item()
    wf = fused.gemm(wcat, w_in.contiguous(), False, False)
    print("wf", err(wf, wcat.double() @ w_in.double(), wcat.abs().double() @ w_in.abs().double()))
    bf = fused.gemm(wcat, b_in.contiguous().view(-1, 1), False, False).view(-1)
    print("bf", err(bf, wcat.double() @ b_in.double(), wcat.abs().double() @ b_in.abs().double()))


if __name__ == "__main__" and os.environ.get("FOLD_WEIGHTS_CHECK"):
    weight_products()


def bisect(name="GraphSage_addAggr_Shared"):
    """Which folded weight product moves the gradients: route one group of them at a time to
    torch.mm (by shape) and report the mean relative error against fp64."""
    dev = torch.device("cuda", 0)
    orig = fused.gemm
    groups = {"none": set(), "wf,bf": {(1024, 128, 512), (1024, 1, 512)}, "dw": {(1024, 512, 128)},
              "dw_in,db_in": {(512, 128, 1024), (512, 1, 1024)}}

    def make(route):
        def g(a, b, trans_a, trans_b, **kw):
            M = a.size(1) if trans_a else a.size(0)
            K = a.size(0) if trans_a else a.size(1)
            N = b.size(0) if trans_b else b.size(1)
            if (M, N, K) in route and not kw:
                return torch.mm(a.t() if trans_a else a, b.t() if trans_b else b)
            return orig(a, b, trans_a, trans_b, **kw)
        return g
    fused.FOLD_WEIGHTS_TORCH = False
    out = {}
    for gname, route in groups.items():
        fused.gemm = make(route)
        b, sd, _, g = T.run(dev, name, 512, True)
        out[gname] = g
    fused.gemm = orig
    exact = T.oracle_grads(b, sd, name)
    for gname, g in out.items():
        errs = [T.rel_err(g[k], exact[k]) for k in exact]
        print(f"torch for {gname:12s}: mean rel err {sum(errs) / len(errs):.2e} max {max(errs):.2e}")


if __name__ == "__main__" and os.environ.get("FOLD_BISECT"):
    bisect()


def inmodel(name="GraphSage_addAggr_Shared"):
    """bgnn vs fp64 for the folded forward products as called inside the model."""
    dev = torch.device("cuda", 0)
    orig = fused.gemm

    def g(a, b, trans_a, trans_b, **kw):
        c = orig(a, b, trans_a, trans_b, **kw)
        M = a.size(1) if trans_a else a.size(0)
        N = b.size(0) if trans_b else b.size(1)
        if M <= 1024 and N <= 1024:
            A = a.double().t() if trans_a else a.double()
            B = b.double().t() if trans_b else b.double()
            torch.cuda.synchronize()
            r = A @ B
            e = ((c.double() - r).abs() / (A.abs() @ B.abs()).clamp_min(1e-300)).max().item()
            l2 = ((c.double() - r).norm() / r.norm().clamp_min(1e-300)).item()
            print(f"  gemm {tuple(a.shape)} x {tuple(b.shape)} ta={trans_a} tb={trans_b}: max/(|A||B|) {e:.2e}"
                  f" rel L2 {l2:.2e}  ||C|| / || |A||B| || {(r.norm() / (A.abs() @ B.abs()).norm()).item():.2e}",
                  flush=True)
        return c
    fused.gemm = g
    T.run(dev, name, 512, True)
    fused.gemm = orig


if __name__ == "__main__" and os.environ.get("FOLD_INMODEL"):
    inmodel()


def relu_flips(name="GraphSage_addAggr_Shared"):
    """Layer outputs x_next of the folded path with Wf, bf on bgnn vs on torch.mm: how many
    elements sit on different sides of ReLU's kink (x_next == 0 in one run, > 0 in the other)."""
    from bgnn import buckgnn
    dev = torch.device("cuda", 0)
    orig_layer, orig_gemm = buckgnn.sage_layer, fused.gemm
    outs = {}

    def rec(tag):
        def f(*a, **kw):
            r = orig_layer(*a, **kw)
            outs.setdefault(tag, []).append((r[0] if isinstance(r, tuple) else r).detach().clone())
            return r
        return f

    def torch_small(a, b, trans_a, trans_b, **kw):
        M = a.size(1) if trans_a else a.size(0)
        N = b.size(0) if trans_b else b.size(1)
        if M <= 1024 and N <= 128 and not kw:
            return torch.mm(a.t() if trans_a else a, b.t() if trans_b else b)
        return orig_gemm(a, b, trans_a, trans_b, **kw)
    for tag in ("bgnn", "torch"):
        buckgnn.sage_layer = rec(tag)
        fused.gemm = torch_small if tag == "torch" else orig_gemm
        T.run(dev, name, 512, True)
    buckgnn.sage_layer, fused.gemm = orig_layer, orig_gemm
    for i, (u, v) in enumerate(zip(outs["bgnn"], outs["torch"])):
        flips = int(((u == 0) != (v == 0)).sum())
        rel = ((u - v).norm() / v.norm()).item()
        print(f"layer {i}: x_next rel diff {rel:.2e}, ReLU side flips {flips} of {u.numel()}")


if __name__ == "__main__" and os.environ.get("FOLD_FLIPS"):
    relu_flips()


def m16_bisect(name="GraphSage_addAggr_Shared"):
    """Which GEMM call of the folded path moves its gradients when it runs on 16x16x32 MFMAs: with
    the product library (4-wave 128x128 tile = 32x32x16, 8-wave tiles = 16x16x32), force the 8-wave
    256x128 tile (bgnn_gemm_set_cfg 1) for one group of fused.gemm calls at a time, identified by
    (M, N, K, trans_a, trans_b), and report the gradients' mean / max relative error against fp64.
    The folded layer's calls at the test batch (4 x 24x24 meshes, N = 2304 rows, H = 512,
    K_in = 128): fwd_fold z = h Wf^T + bf; dgrad_fold dh = dz Wf; wgrad_fold dWf = dz^T h; and the
    weight products wf, bf, dw, dw_in, db_in."""
    from bgnn import _lib
    dev = torch.device("cuda", 0)
    orig = fused.gemm
    N, H, K = 2304, 512, 128
    groups = {"none": set(),
              "fwd_fold": {(N, 2 * H, K, False, True)}, "dgrad_fold": {(N, K, 2 * H, False, True)},
              "wgrad_fold": {(2 * H, K, N, True, False)},
              "wf": {(2 * H, K, H, False, False)}, "bf": {(2 * H, 1, H, False, False)},
              "dw": {(2 * H, H, K, False, True)}, "dw_in": {(H, K, 2 * H, True, False)},
              "db_in": {(H, 1, 2 * H, True, False)}}
    groups["all"] = set().union(*groups.values())
    seen = set()

    def make(route):
        def g(a, b, trans_a, trans_b, **kw):
            M = a.size(1) if trans_a else a.size(0)
            Kd = a.size(0) if trans_a else a.size(1)
            Nn = b.size(0) if trans_b else b.size(1)
            key = (M, Nn, Kd, bool(trans_a), bool(trans_b))
            seen.add(key)
            if key in route:
                _lib.call("bgnn_gemm_set_cfg", 1)
                try:
                    return orig(a, b, trans_a, trans_b, **kw)
                finally:
                    _lib.call("bgnn_gemm_set_cfg", -1)
            return orig(a, b, trans_a, trans_b, **kw)
        return g
    fused.FOLD_WEIGHTS_TORCH = False
    out = {}
    for gname, route in groups.items():
        fused.gemm = make(route)
        b, sd, _, g = T.run(dev, name, 512, True)
        out[gname] = g
    fused.gemm = orig
    exact = T.oracle_grads(b, sd, name)
    print("fused.gemm calls seen (M, N, K, ta, tb):", sorted(seen))
    for gname, g in out.items():
        errs = [T.rel_err(g[k], exact[k]) for k in exact]
        print(f"16x16x32 for {gname:10s}: mean rel err {sum(errs) / len(errs):.2e} max {max(errs):.2e}", flush=True)


if __name__ == "__main__" and os.environ.get("FOLD_M16_BISECT"):
    m16_bisect()


def global_cfg(name="GraphSage_addAggr_Shared"):
    """Folded and unfolded gradients against fp64 (mean / max relative error over parameters) with
    every bgnn GEMM of the step on its planned tile (-1: the 4-wave 128x128 tile of these N = 2304
    shapes runs 32x32x16 MFMAs) or forced onto the 8-wave 256x128 tile (1: 16x16x32 MFMAs), for
    three weight seeds: whether a change of MFMA shape moves the folded path's error systematically
    or only reshuffles which rounding-sensitive elements the comparison meets."""
    import bgnn
    from bgnn import _lib, buckgnn
    from bgnn import synthetic as S
    dev = torch.device("cuda", 0)
    b = S.make_batch(24, 4)

    def run(seed, fold):
        torch.manual_seed(seed)
        m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name=name)
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        m = m.to(dev).train()
        old = buckgnn.FOLD_ENCODER
        buckgnn.FOLD_ENCODER = fold
        try:
            bd = b.to(dev)
            pred, _ = m(bd.x, bd.edge_index, bd.edge_attr, bd.batch)
            bgnn.RelativeErrorLoss()(pred, bd.y).backward()
        finally:
            buckgnn.FOLD_ENCODER = old
        return sd, {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    for seed in (0, 1, 2):
        exact = None
        for cfg in (-1, 1):
            _lib.call("bgnn_gemm_set_cfg", cfg)
            try:
                res = {f: run(seed, f) for f in (False, True)}
            finally:
                _lib.call("bgnn_gemm_set_cfg", -1)
            if exact is None:
                exact = T.oracle_grads(b, res[False][0], name)
            line = []
            for f in (False, True):
                errs = [T.rel_err(res[f][1][k], exact[k]) for k in exact]
                line.append(f"{'folded' if f else 'unfolded'} mean {sum(errs) / len(errs):.2e} max {max(errs):.2e}")
            print(f"seed {seed} gemm cfg {cfg:2d} ({'32x32x16' if cfg < 0 else '16x16x32'} at N = 2304): "
                  + " | ".join(line), flush=True)


if __name__ == "__main__" and os.environ.get("FOLD_GLOBAL_CFG"):
    global_cfg()
