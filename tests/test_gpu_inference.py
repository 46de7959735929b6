"""opt_runs.run_inference_queue (opt_runs.py:560-646) as a drop-in: the q x seed
RedQueen grid, and after every Opt replica the Poisson follow-up at its capacity
and the Oracle follow-up at that capacity.

Parity: every Opt and Poisson row equals the engine-semantics oracle
(oracle/rq_oracle.c) on that replica's world bit for bit; every Oracle row equals
the single worker_oracle call (whose DP + replay are pinned to the reference's
worker_oracle outputs in tests/golden/oracle.npz, test_gpu_analysis.py); the
batched Opt/Poisson legs equal the per-replica worker path; the returned
Options(df, raw_results, capacities) has the reference's fields."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from redqueen_amd import opt_runs as R
    from redqueen_amd.opt_model import SimOpts
    return O, R, SimOpts


def _gen(SimOpts):
    def gen(seed):
        return SimOpts.std_poisson(world_rate=4.0, world_seed=seed + 42).update({"end_time": 20.0})
    return gen


def _check_against_oracle(O, R, out, gen, N, T, Ks=(1,)):
    df = out.df
    assert list(df.columns) == R.perf_opts.performance_fields
    qs = np.logspace(-1, 3, num=10)
    assert sorted(out.capacities) == sorted(qs)
    for q in qs:
        assert [s for s, _ in out.capacities[q]] == list(range(N))
    opt = {(r["q"], r["seed"]): r for r in out.raw_results if r["type"] == "Opt"}
    poi = {(r["q"], r["seed"]): r for r in out.raw_results if r["type"] == "Poisson"}
    orc = {(r["q"], r["seed"]): r for r in out.raw_results if r["type"] == "Oracle"}
    assert len(opt) == len(poi) == 10 * N
    for (q, seed), r in opt.items():
        so = gen(seed).update({"q": q})
        (top, avg, r2, cnt), _ = O.engine_metrics(O.Scenario(so.get_dict(), ("opt", seed)), Ks)
        assert (r["top_1"], r["avg_rank"], r["r_2"], r["num_events"], r["world_events"]) == \
            (top[0], avg, r2, cnt[0], cnt[1]), (q, seed)
        assert r["capacity"] == float(cnt[0])
        assert r["wall_intensities"].shape[0] == len(so.sink_ids)
        p = poi[(q, seed)]
        (top, avg, r2, cnt), _ = O.engine_metrics(
            O.Scenario(so.get_dict(), ("poisson", seed, r["capacity"] / T)), Ks)
        assert (p["top_1"], p["avg_rank"], p["r_2"], p["num_events"]) == (top[0], avg, r2, cnt[0])
    # the Oracle rows: those whose worker_oracle does not raise, equal to it
    for (q, seed), r in opt.items():
        so = gen(seed).update({"q": q})
        try:
            want = R.worker_oracle((seed, r["capacity"], r["world_events"], so, None))
        except Exception:
            assert (q, seed) not in orc
            continue
        got = orc[(q, seed)]
        for k in ("top_1", "avg_rank", "r_2", "num_events", "world_events", "r0_num_events"):
            assert got[k] == want[k], (q, seed, k)
    return opt, poi, orc


def test_run_inference_queue_batched():
    O, R, SimOpts = _ctx()
    gen = _gen(SimOpts)
    N = 3
    out = R.run_inference_queue(N=N, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3,
                                log_q_low=-1)
    opt, poi, orc = _check_against_oracle(O, R, out, gen, N, 20.0)
    assert len(orc) > 0
    assert len(out.df) == len(opt) + len(poi) + len(orc)


def test_run_inference_equals_queue_legs(caplog):
    """opt_runs.run_inference (opt_runs.py:350-440): the Opt / Poisson / Oracle legs of the
    q x seed sweep -- the same records as run_inference_queue, without the Karimi leg the
    reference's run_inference has commented out."""
    import logging
    O, R, SimOpts = _ctx()
    gen = _gen(SimOpts)
    a = R.run_inference_queue(N=2, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
    caplog.clear()
    with caplog.at_level(logging.ERROR):
        b = R.run_inference(N=2, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
    assert a.df.equals(b.df) and set(a.capacities) == set(b.capacities)
    assert not any("kdd" in r.getMessage() for r in caplog.records)
    _check_against_oracle(O, R, b, gen, 2, 20.0)


def test_batched_equals_per_replica_workers(monkeypatch):
    """The two-batch Opt/Poisson legs == one worker_opt / worker_poisson per replica."""
    O, R, SimOpts = _ctx()
    gen = _gen(SimOpts)
    a = R.run_inference_queue(N=2, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
    monkeypatch.setattr(R, "_randomize_seed", lambda so: None)   # force the per-replica path
    b = R.run_inference_queue(N=2, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
    assert a.df.equals(b.df)
    for x, y in zip(a.raw_results, b.raw_results):
        if x["type"] == "Opt":
            assert np.array_equal(x["wall_intensities"], y["wall_intensities"], equal_nan=True)


def test_two_source_world_unbatchable():
    """Worlds whose seeds are not randomize_other_sources seeds run replica by replica;
    a multi-follower world's Oracle tasks raise (oracle_ranking's one-follower
    assert) and are dropped, as the reference's queue drops exception records."""
    O, R, SimOpts = _ctx()

    def gen(seed):
        return SimOpts(src_id=1, end_time=15.0, q=1.0, s=1.0, sink_ids=[7, 8],
                       other_sources=[("Poisson2", {"src_id": 2, "seed": 3 * seed + 1, "rate": 2.0}),
                                      ("Hawkes", {"src_id": 3, "seed": 5 * seed + 2, "l_0": 1.0,
                                                  "alpha": 1.0, "beta": 5.0})],
                       edge_list=[(1, 7), (1, 8), (2, 7), (3, 7), (3, 8)])
    assert R._randomize_seed(gen(1)) is None
    out = R.run_inference_queue(N=2, T=15.0, num_segments=3, sim_opts_gen=gen, log_q_high=3, log_q_low=-1)
    opt, poi, orc = _check_against_oracle(O, R, out, gen, 2, 15.0)
    assert len(orc) == 0


def test_reference_configs_exist():
    O, R, SimOpts = _ctx()
    for o in (R.poisson_inf_opts, R.hawkes_inf_opts, R.piecewise_inf_opts):
        so = o.sim_opts_gen(3)
        assert so.end_time == R.simulation_opts.T and R._randomize_seed(so) is not None


def test_per_seed_significance_unbatchable():
    """worlds that differ only in the followers' significance s must not
    share one batch (the batch runs one s); each replica then runs its own s, and every
    row still equals the engine oracle on that replica's own SimOpts."""
    O, R, SimOpts = _ctx()
    base = _gen(SimOpts)

    def gen(seed):
        return base(seed).update({"s": np.asarray([1.0 + seed])})
    assert R._world_key(gen(0)) != R._world_key(gen(1))
    assert R._world_key(base(0)) == R._world_key(base(1))
    out = R.run_inference_queue(N=2, T=20.0, num_segments=4, sim_opts_gen=gen, log_q_high=3,
                                log_q_low=-1)
    _check_against_oracle(O, R, out, gen, 2, 20.0)


def test_oracle_batch_equals_single_searches():
    """utils.find_opt_oracle_batch (every search in lockstep, one DP launch per round)
    returns what find_opt_oracle returns search by search."""
    O, R, SimOpts = _ctx()
    from redqueen_amd import utils as U
    gen = _gen(SimOpts)
    sos = [gen(s).update({"q": q}) for s in range(3) for q in (0.1, 10.0)]
    targets = [3.0, 7.0, 12.0, 2.0, 5.0, 9.0]
    got = U.find_opt_oracle_batch(targets, sos, [None] * len(sos))
    for t, so, g in zip(targets, sos, got):
        want = U.find_opt_oracle(t, so)
        assert set(g) == set(want) and g["q"] == want["q"] and g["cost"] == want["cost"]
        key = "df" if "df" in g else "oracle_df"
        assert g[key].equals(want[key])
