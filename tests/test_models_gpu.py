"""End-to-end model numerics on the MI355X: one forward+backward of every
model family through the HIP kernels vs the fp32 PyTorch reference path of
the same ops (same seed, same synthetic batch), plus a few training steps."""
import math

import pytest
import torch

from tiresias_amd.executor.trainer import Trainer

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.fixture(autouse=True)
def _production_policies(gpu):
    """Model-level parity is claimed for the configuration production runs:
    every kernel policy must hold its load-time (production) value here,
    whatever kernel tests ran before (conftest restores them after each)."""
    import conftest

    names = str(torch.ops.tam.policy_names()).split(",")
    state = conftest.policy_state()
    diff = {n: (v, p) for n, v, p in zip(names, state, conftest.PRODUCTION_POLICIES) if v != p}
    assert not diff, f"non-production kernel policies at model test start: {diff}"


@pytest.mark.parametrize("model", ["resnet_tiny", "vgg_tiny", "transformer_tiny", "gnmt_tiny"])
def test_model_grads_match_reference(gpu, model):
    tg = Trainer(model, gpu, seed=3)
    tc = Trainer(model, "cpu", seed=3)
    # same initial weights (device RNG streams differ between CPU and GPU)
    tc.arena.master.copy_(tg.arena.master.cpu())
    tc.arena.shadow.copy_(tg.arena.shadow.cpu())
    tc.data = {k: v.cpu() for k, v in tg.data.items()}
    lg = tg._fwd_bwd()
    lc = tc._fwd_bwd()
    assert abs(float(lg) - float(lc)) < 0.02 * max(1.0, abs(float(lc)))
    e = rel(tg.arena.grad.cpu(), tc.arena.grad)
    assert e < 0.05, f"{model}: grad rel err {e}"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model,batch", [("transformer", 8), ("gnmt", 16)])
def test_full_size_grads_match_reference(gpu, model, batch):
    """Full-size Transformer-base and GNMT (hidden 1024, 4+4 layers; the
    persistent LSTM recurrence runs at B = 16) vs the fp32 PyTorch path of
    the same ops on the host: one eager forward+backward from identical
    weights and batch. (Small batch keeps the fp32 host reference to
    seconds; the architecture is the full one.)"""
    torch.manual_seed(0)
    tg = Trainer(model, gpu, seed=3, batch=batch)
    tc = Trainer(model, "cpu", seed=3, batch=batch)
    tc.arena.master.copy_(tg.arena.master.cpu())
    tc.arena.shadow.copy_(tg.arena.shadow.cpu())
    tc.data = {k: v.cpu() for k, v in tg.data.items()}
    lg = tg._fwd_bwd()
    torch.cuda.synchronize()
    lc = tc._fwd_bwd()
    assert abs(float(lg) - float(lc)) < 0.02 * max(1.0, abs(float(lc)))
    gg, gc = tg.arena.grad.cpu(), tc.arena.grad
    e = rel(gg, gc)
    assert e < 0.05, f"{model}: grad rel err {e}"
    # every parameter tensor, not only the global norm
    floor = 1e-4 * float(gc.norm())      # parameters with a non-negligible gradient
    worst = max((rel(gg[p.offset:p.offset + p.numel], gc[p.offset:p.offset + p.numel]), p.name)
                for p in tg.arena.params if float(gc[p.offset:p.offset + p.numel].norm()) > floor)
    assert worst[0] < 0.1, f"{model}: worst parameter {worst[1]} rel err {worst[0]}"
    if model == "gnmt":
        from tiresias_amd.models import gnmt as G

        assert G.persist_errors() == 0


@pytest.mark.parametrize("model", ["resnet_tiny", "transformer_tiny", "gnmt_tiny", "vgg_tiny"])
def test_model_trains(gpu, model):
    t = Trainer(model, gpu, seed=1)
    losses = [float(t.step()) for _ in range(8)]
    assert losses[-1] < losses[0]
    assert all(l == l for l in losses)   # no NaN


def test_graph_capture_matches_eager(gpu):
    a = Trainer("resnet_tiny", gpu, seed=5, use_graph=True)
    b = Trainer("resnet_tiny", gpu, seed=5, use_graph=False)
    for _ in range(3):
        la = float(a.step())
        lb = float(b.step())
    assert abs(la - lb) < 1e-2 * max(1.0, abs(lb))
    assert rel(a.arena.master, b.arena.master) < 1e-3


@pytest.mark.parametrize("model", ["resnet_tiny", "vgg_tiny", "transformer_tiny", "gnmt_tiny"])
def test_wgrad_stream_overlap_matches(gpu, model):
    """Weight gradients issued on the side stream (ops/functional.py
    set_wgrad_stream; tied embedding/projection writers included) give the
    same gradients as the single-stream backward, eager and under capture."""
    a = Trainer(model, gpu, seed=4, overlap_wgrad=True)
    b = Trainer(model, gpu, seed=4, overlap_wgrad=False)
    b.arena.master.copy_(a.arena.master)
    b.arena.shadow.copy_(a.arena.shadow)
    la, lb = a._fwd_bwd(), b._fwd_bwd()
    torch.cuda.synchronize()
    assert abs(float(la) - float(lb)) < 1e-3 * max(1.0, abs(float(lb)))
    assert rel(a.arena.grad, b.arena.grad) < 1e-3
    g = Trainer(model, gpu, seed=4, overlap_wgrad=True, use_graph=True)
    e = Trainer(model, gpu, seed=4, overlap_wgrad=False, use_graph=False)
    for _ in range(4):
        lg, le = float(g.step()), float(e.step())
    assert abs(lg - le) < 2e-2 * max(1.0, abs(le))


@pytest.mark.parametrize("overlap", [True, False])
def test_grouped_wgrad_matches(gpu, overlap, monkeypatch):
    """Transformer (full width, 2+2 layers) with every Linear weight gradient
    deferred into the grouped launch gives the gradients of the per-layer
    path, eager and under hipGraph capture, with and without the weight-
    gradient stream, and with a mid-backward chunked flush."""
    from tiresias_amd.ops import functional as Fx

    kw = dict(enc_layers=2, dec_layers=2)
    a = Trainer("transformer", gpu, seed=4, batch=4, model_kwargs=kw, overlap_wgrad=overlap)
    b = Trainer("transformer", gpu, seed=4, batch=4, model_kwargs=kw, overlap_wgrad=overlap)
    assert a.group_wgrad
    b.group_wgrad = False
    b.arena.master.copy_(a.arena.master)
    b.arena.shadow.copy_(a.arena.shadow)
    calls = []
    real = Fx.flush_wgrad
    monkeypatch.setattr(Fx, "flush_wgrad", lambda: calls.append(real()) or calls[-1])
    la, lb = a._fwd_bwd(), b._fwd_bwd()
    torch.cuda.synchronize()
    assert calls and calls[0] >= 20, calls         # the Linear layers went through the group
    assert abs(float(la) - float(lb)) < 1e-3 * max(1.0, abs(float(lb)))
    assert rel(a.arena.grad, b.arena.grad) < 2e-3
    monkeypatch.setattr(Fx, "_DEFER_CHUNK", 5)     # flushes every 5 deferred layers
    a.arena.grad.zero_()
    a._fwd_bwd()
    torch.cuda.synchronize()
    assert rel(a.arena.grad, b.arena.grad) < 2e-3
    monkeypatch.setattr(Fx, "_DEFER_CHUNK", 0)
    g = Trainer("transformer", gpu, seed=4, batch=4, model_kwargs=kw, overlap_wgrad=overlap, use_graph=True)
    e = Trainer("transformer", gpu, seed=4, batch=4, model_kwargs=kw, overlap_wgrad=overlap)
    e.group_wgrad = False
    e.arena.master.copy_(g.arena.master)
    e.arena.shadow.copy_(g.arena.shadow)
    for _ in range(4):
        lg, le = float(g.step()), float(e.step())
    assert abs(lg - le) < 2e-2 * max(1.0, abs(le))
    assert rel(g.arena.master, e.arena.master) < 1e-3


@pytest.mark.timeout(300)
def test_resnet50_grouped_conv_wgrad_matches(gpu, monkeypatch):
    """ResNet-50 (full size, batch 32): the 1x1 stride-1 conv weight
    gradients deferred into the grouped launch (K-split over the output
    pixels, fp32 atomics between slices) give the per-conv path's gradients,
    eager and under hipGraph replay."""
    from tiresias_amd.ops import functional as Fx

    a = Trainer("resnet50", gpu, seed=6, batch=32)
    b = Trainer("resnet50", gpu, seed=6, batch=32)
    assert a.group_wgrad
    b.group_wgrad = False
    b.arena.master.copy_(a.arena.master)
    b.arena.shadow.copy_(a.arena.shadow)
    calls = []
    real = Fx.flush_wgrad
    monkeypatch.setattr(Fx, "flush_wgrad", lambda: calls.append(real()) or calls[-1])
    la, lb = a._fwd_bwd(), b._fwd_bwd()
    torch.cuda.synchronize()
    assert calls and calls[0] >= 20, calls          # the 1x1 convs of stages 1-3 went through the group
    assert abs(float(la) - float(lb)) < 1e-3 * max(1.0, abs(float(lb)))
    assert rel(a.arena.grad, b.arena.grad) < 2e-3
    # second backward (the deferred-problem count is stable step to step)
    a.arena.grad.zero_()
    a._fwd_bwd()
    torch.cuda.synchronize()
    assert a._defer_n == calls[0] and len(calls) == 2 and calls[1] == calls[0], calls
    assert rel(a.arena.grad, b.arena.grad) < 2e-3
    monkeypatch.setattr(Fx, "flush_wgrad", real)
    g = Trainer("resnet50", gpu, seed=6, batch=32, use_graph=True)
    e = Trainer("resnet50", gpu, seed=6, batch=32)
    e.group_wgrad = False
    e.arena.master.copy_(g.arena.master)
    e.arena.shadow.copy_(g.arena.shadow)
    for _ in range(4):
        lg, le = float(g.step()), float(e.step())
    assert abs(lg - le) < 2e-2 * max(1.0, abs(le))
    assert rel(g.arena.master, e.arena.master) < 1e-3


def test_gnmt_lstm_grouped_wgrad_matches(gpu, monkeypatch):
    """GNMT's per-layer LSTM weight gradients (dW_hh, dW_ih + the bias column
    sums) as one grouped launch (models/gnmt.py LSTM_GROUPED_WGRAD, store-
    mode first writes) give the gradients and the training trajectory of the
    per-GEMM path (batch 64, so every layer's problems are grouped)."""
    import tiresias_amd.models.gnmt as G
    kw = dict(hidden=256, enc_layers=3, dec_layers=2, heads=4)      # the batch's 32000-token vocabulary
    runs = []
    # (grouped, deferred into the backward's one launch): deferred (the
    # production path), one grouped launch per layer, per-GEMM (reference)
    for grouped, defer in ((True, True), (True, False), (False, False)):
        monkeypatch.setattr(G, "LSTM_GROUPED_WGRAD", grouped)
        monkeypatch.setattr(G, "LSTM_DEFER_WGRAD", defer)
        t = Trainer("gnmt", gpu, seed=8, batch=64, model_kwargs=kw)
        loss = float(t._fwd_bwd())
        torch.cuda.synchronize()
        grad = t.arena.grad.clone()
        t.arena.grad.zero_()
        losses = [float(t.step()) for _ in range(3)]
        torch.cuda.synchronize()
        runs.append((loss, grad, losses, t.arena.master.clone()))
    lb, gb, lsb, mb = runs[-1]
    for la, ga, lsa, ma in runs[:-1]:
        assert abs(la - lb) < 1e-4 * max(1.0, abs(lb))
        assert rel(ga, gb) < 2e-3
        assert all(abs(x - y) < 1e-2 * max(1.0, abs(y)) for x, y in zip(lsa, lsb)), (lsa, lsb)
        assert rel(ma, mb) < 1e-3


@pytest.mark.parametrize("overlap", [False, True])
def test_gnmt_branch_streams_match(gpu, overlap):
    """GNMT's independent recurrences on branch streams (bidirectional
    halves; first decoder layer alongside the encoder; ops/functional.py
    on_branch) give the same loss and gradients as the one-stream order,
    eager and under hipGraph capture, with and without the wgrad stream."""
    a = Trainer("gnmt_tiny", gpu, seed=6, branches=True, overlap_wgrad=overlap)
    b = Trainer("gnmt_tiny", gpu, seed=6, branches=False, overlap_wgrad=overlap)
    b.arena.master.copy_(a.arena.master)
    b.arena.shadow.copy_(a.arena.shadow)
    for _ in range(2):
        la, lb = a._fwd_bwd(), b._fwd_bwd()
        torch.cuda.synchronize()
        assert abs(float(la) - float(lb)) < 1e-3 * max(1.0, abs(float(lb)))
        assert rel(a.arena.grad, b.arena.grad) < 1e-3
        a.arena.grad.zero_()
        b.arena.grad.zero_()
    g = Trainer("gnmt_tiny", gpu, seed=6, branches=True, overlap_wgrad=overlap, use_graph=True)
    e = Trainer("gnmt_tiny", gpu, seed=6, branches=False, overlap_wgrad=overlap, use_graph=False)
    for _ in range(5):
        lg, le = float(g.step()), float(e.step())
    torch.cuda.synchronize()
    assert abs(lg - le) < 2e-2 * max(1.0, abs(le))
    assert rel(g.arena.master, e.arena.master) < 1e-3


@pytest.mark.parametrize("model", ["vgg_tiny", "gnmt_tiny", "transformer"])
@pytest.mark.parametrize("graph", [False, True])
def test_store_grad_matches_accumulate(gpu, model, graph, monkeypatch):
    """store_grad weights (first gradient write of a step stores, the
    optimizer skips zeroing them; ops/functional.py grad_mode) train exactly
    like the zero-then-accumulate path over several optimizer steps, eager
    and under hipGraph replay."""
    import tiresias_amd.ops.functional as Fx
    runs = []
    for store in (True, False):
        monkeypatch.setattr(Fx, "STORE_GRAD", store)
        kw = dict(enc_layers=2, dec_layers=2) if model == "transformer" else None
        t = Trainer(model, gpu, seed=7, use_graph=graph, batch=4 if model == "transformer" else None,
                    model_kwargs=kw)
        assert any(p.store_grad for p in t.arena.params) and t.arena.n_store > 0
        losses = [float(t.step()) for _ in range(5)]
        torch.cuda.synchronize()
        runs.append((losses, t.arena.master.clone()))
    (la, ma), (lb, mb) = runs
    assert all(abs(x - y) < 1e-3 * max(1.0, abs(y)) for x, y in zip(la, lb)), (la, lb)
    assert rel(ma, mb) < 1e-4


def test_ddp_bucket_event_timing(gpu, monkeypatch):
    """GradBucketer records hipEvents around every step's gradient sync and
    poll_timing() turns finished steps into exposed / span seconds (a
    stand-in 2-rank comm: the event plumbing, not RCCL, is under test)."""
    from tiresias_amd.ops.arena import Arena
    from tiresias_amd.parallel import ddp as D

    class FakeComm:
        def start(self, view):
            view.mul_(2.0)
            return None

        def finish(self, works):
            pass

    monkeypatch.setattr(D.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(D, "as_comm", lambda g: g)
    monkeypatch.setattr(D, "comm_size", lambda c: 2)
    A = Arena(gpu)
    p = A.add("w", (4096, 1024))
    A.materialize()
    b = D.GradBucketer(A, FakeComm(), bucket_mb=4)
    for _ in range(3):
        A.grad.fill_(1.0)
        p.grad_ready()
        b.finish()
    torch.cuda.synchronize()
    t = b.poll_timing()
    assert t["steps"] == 3 and t["span_s"] >= t["exposed_s"] >= 0.0
    assert b.poll_timing()["steps"] == 0


def test_kernel_debug_mode_names_the_op(gpu, monkeypatch):
    """utils/debug.py: per-op synchronisation + NaN/Inf check of the outputs
    names the op that produced non-finite values; trainers run eagerly."""
    from tiresias_amd.ops import _lib
    from tiresias_amd.utils import debug

    monkeypatch.setattr(debug, "_LEVEL", 2)
    T = _lib.ops()
    assert isinstance(T, debug.OpsProxy)
    a = torch.randn(64, 64, device=gpu).to(torch.bfloat16)
    b = torch.randn(64, 64, device=gpu).to(torch.bfloat16)
    c = torch.empty(64, 64, device=gpu)
    T.gemm(a, True, b, True, c, 0, None, False, None, 1.0, False)      # clean op passes
    a[3, 5] = float("inf")
    with pytest.raises(debug.KernelDebugError, match="tam.gemm"):
        T.gemm(a, True, b, True, c, 0, None, False, None, 1.0, False)
    t = Trainer("resnet_tiny", gpu, seed=1, use_graph=True)
    assert not t.use_graph                      # capture + per-op sync do not mix
    assert math.isfinite(float(t.step()))


@pytest.mark.timeout(300)
def test_persist_barrier_timeout_is_loud_and_falls_back(gpu):
    """A persistent-LSTM grid barrier that times out (forced: poll bound 1)
    must not pass silently: the worker reads the sticky device counter after
    the round's synchronize, reports a PersistTimeout error for the job and
    switches it to the per-step recurrence; the next round runs clean (no
    timeouts, finite loss, per-step path)."""
    from tiresias_amd.executor.cluster_runtime import Worker
    from tiresias_amd.models import gnmt as G
    from tiresias_amd.ops import _lib

    T = _lib.ops()
    w = Worker(0, 1, gpu, monitor_period=0)
    start = {"op": "start", "job": "1", "model": "gnmt", "batch": 16, "seed": 1, "ranks": (0,), "source": "fresh"}
    w.apply({"actions": [start], "assign": {}})
    assert w.trainers["1"].uses_persist
    G.device_timeouts(reset=True)
    T.lstm_seq_spin_limit(1)
    try:
        rep = w.run({"actions": [], "assign": {0: [("1", 1)]}, "deadline": None})
    finally:
        T.lstm_seq_spin_limit(0)
    err = rep["jobs"][0].get("error") or ""
    assert "PersistTimeout" in err, rep
    assert rep["jobs"][0]["iters"] == 0, rep        # the guarded step is not progress
    assert not w.trainers["1"].model.persist
    assert int(w.trainers["1"].model.err.sum()) == 0      # read and reset by the worker
    assert G.device_timeouts(reset=True) > 0              # the device-wide counter saw them too
    rep2 = w.run({"actions": [], "assign": {0: [("1", 2)]}, "deadline": None})
    assert "error" not in rep2["jobs"][0], rep2
    assert rep2["jobs"][0]["iters"] == 2
    assert rep2["jobs"][0]["loss"] == rep2["jobs"][0]["loss"]          # finite
    assert G.device_timeouts(reset=False) == 0
    assert w.trainers["1"].persist_skipped(reset=False) == 0
    w.clear(keep_pool=False)


def test_two_persistent_jobs_sharing_a_gpu_run_per_step(gpu):
    """GPU sharing with two GNMT jobs: their persistent LSTM grids (different
    kernels, different per-CU footprints) cannot be guaranteed co-resident, so
    a shared round switches both to the per-step recurrence before stepping;
    the round completes with finite losses and no barrier timeouts."""
    from tiresias_amd.executor.cluster_runtime import Worker
    from tiresias_amd.models import gnmt as G

    w = Worker(0, 1, gpu, monitor_period=0)
    acts = [{"op": "start", "job": j, "model": "gnmt", "batch": 16, "seed": int(j), "ranks": (0,),
             "source": "fresh"} for j in ("1", "2")]
    w.apply({"actions": acts, "assign": {}})
    assert w.trainers["1"].uses_persist and w.trainers["2"].uses_persist
    G.device_timeouts(reset=True)
    rep = w.run({"actions": [], "assign": {0: [("1", 2), ("2", 2)]}, "deadline": None})
    for r in rep["jobs"]:
        assert "error" not in r and r["iters"] == 2 and r["shared"], rep
        assert r["loss"] == r["loss"]                                   # finite
    assert not w.trainers["1"].uses_persist and not w.trainers["2"].uses_persist
    assert G.device_timeouts(reset=False) == 0
    # alone again: back on the persistent grids (the switch is per round,
    # not for good -- only a barrier timeout turns them off for good)
    rep = w.run({"actions": [], "assign": {0: [("1", 2)]}, "deadline": None})
    assert rep["jobs"][0]["iters"] == 2 and "error" not in rep["jobs"][0], rep
    assert w.trainers["1"].uses_persist
    assert G.device_timeouts(reset=False) == 0
    w.clear(keep_pool=False)


def test_snapshot_roundtrip_on_device(gpu, tmp_path):
    """ckpt/snapshot.py on the GPU: D2D clone on the compute stream, D2H on
    the low-priority side stream, atomic file; steps issued right after the
    snapshot do not leak into it; a fresh trainer restored from the file
    matches the state (master, optimizer) at the snapshot's step."""
    from tiresias_amd.ckpt.snapshot import SnapshotWriter, load_snapshot

    t = Trainer("transformer_tiny", gpu, seed=5)
    for _ in range(3):
        t.step()
    want_w = t.arena.master.clone()
    want_m = t.opt_state[0].clone()
    w = SnapshotWriter(str(tmp_path), gpu)
    w.snapshot("7", t)
    for _ in range(2):                       # keeps training while the copy drains
        t.step()
    w.flush()
    got = w.poll()
    assert got and got[0][0] == "7" and got[0][1] == 3
    u = Trainer("transformer_tiny", gpu, seed=9)
    assert load_snapshot(got[0][2], u) == 3
    torch.cuda.synchronize()
    assert torch.equal(u.arena.master, want_w) and torch.equal(u.opt_state[0], want_m)
    assert not torch.equal(u.arena.master, t.arena.master)
    assert torch.equal(u.arena.shadow, want_w.to(torch.bfloat16))
    w.close()


def test_optimizer_guard_is_per_job(gpu):
    """The persistent-LSTM guard is the JOB's own word: a set guard turns
    that job's optimizer step into a gradient reset and lstm_guard_step
    moves it into the job's skipped-step count; a job with a clear word
    (sharing the device) updates normally."""
    from tiresias_amd.ops import _lib

    T = _lib.ops()
    n = 4096
    for opt in ("sgd", "adam"):
        outs = []
        for bad in (1, 0):
            w = torch.randn(n, device=gpu)
            w0 = w.clone()
            g = torch.randn(n, device=gpu)
            m, v = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
            wb = torch.empty(n, device=gpu, dtype=torch.bfloat16)
            err = torch.tensor([bad, 0], dtype=torch.int32, device=gpu)
            if opt == "sgd":
                T.sgd_step(w, g, m, wb, 0.1, 0.9, 0.0, 1.0, False, True, err)
            else:
                T.adam_step(w, g, m, v, wb, 0.1, 0.9, 0.98, 1e-9, 0.0, 1, 1.0, True, err)
            T.lstm_guard_step(err)
            torch.cuda.synchronize()
            assert float(g.abs().sum()) == 0.0                  # gradient reset either way
            outs.append((torch.equal(w, w0), err.tolist()))
        assert outs[0] == (True, [0, 1]), (opt, outs)           # guarded: no update, counted
        assert outs[1] == (False, [0, 0]), (opt, outs)          # the other job updates
