"""The fused sweep's scheduling knobs change WHEN arrivals are generated and how the
event stream is cut into tiles, never WHAT is computed: every refill policy (forced
refill threshold RQ_FW_HMIN, fill level RQ_FW_HFILL, opportunistic threshold
RQ_FW_THR), ring depth (RQ_FW_W) and tile target (RQ_FW_TILE) must give the same
event log, counts and metrics bit for bit -- and equal the engine oracle.  The knobs
are read by the library at every run (rq_api.cpp), so one process can switch them.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POLICIES = [
    {},                                                      # the defaults
    {"RQ_FW_HMIN": "8", "RQ_FW_HFILL": "16", "RQ_FW_THR": "17"},   # round-2 start: fill to W
    {"RQ_FW_HMIN": "1", "RQ_FW_HFILL": "1", "RQ_FW_THR": "64"},    # laziest: a ring may run dry
    {"RQ_FW_HMIN": "1", "RQ_FW_THR": "1"},                   # eager: a pass for any short ring
    {"RQ_FW_W": "32"},
    {"RQ_FW_W": "8", "RQ_FW_HMIN": "1"},
    {"RQ_FW_TILE": "9"},                                      # short tiles
]


def _run(g, so, env, R, mode=7):
    # sweep_mode 7: the fused sweep generating its arrivals in-kernel (the knobs' subject);
    # the default (mode 0) plays merged pre-generated streams and must agree with it
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return g.run("opt", q=so["q"], s=so["s"], n_rep=R, ctrl_seed=300, world_seed=300,
                     randomize=True, Ks=(1,), event_log=True, sweep_mode=mode)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_refill_policies_same_bits():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redqueen_amd import engine, graphs
    from oracle import oracle as O
    so = graphs.c3()
    g = engine.Graph(so["src_id"], so["other_sources"], so["sink_ids"], so["edge_list"], so["end_time"])
    R = 96
    base = None
    for env in POLICIES + [None]:
        res = _run(g, so, env or {}, R, 7 if env is not None else 0)
        assert int(res.status.max().item()) == 0, env
        got = (res.metrics.cpu().numpy(), res.counts.cpu().numpy(),
               [res.events(i) for i in range(0, R, 5)])
        if base is None:
            base = got
            continue
        assert np.array_equal(got[0], base[0]), env
        assert np.array_equal(got[1], base[1]), env
        for (t, s), (t0, s0) in zip(got[2], base[2]):
            assert np.array_equal(t, t0) and np.array_equal(s, s0), env
    # and the defaults equal the engine oracle on a few replicas (same seeds as
    # randomize_other_sources(u) / create_manager_with_opt(u) with u = 300 + r)
    for r in (0, 41, 95):
        u = 300 + r
        w = dict(so)
        w["other_sources"] = [(n, dict(kw, seed=(u + 99 * i) & 0xFFFFFFFF)) if "seed" in kw else (n, kw)
                              for i, (n, kw) in enumerate(so["other_sources"])]
        met, (t_o, _, s_o) = O.engine_metrics(O.Scenario(w, ("opt", u)), (1,))
        top, avg, r2, _ = met
        assert np.array_equal(base[0][r], np.asarray(list(top) + [avg, r2])), r
