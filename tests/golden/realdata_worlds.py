"""World definitions of tests/golden/realdata.npz (plain data: no reference import),
shared by gen_golden.py and tests/test_gpu_realdata.py."""
import numpy as np


# all-RealData worlds: every source static with given times, so the reference's whole
# df is deterministic and the engine must reproduce it bit for bit (event order with
# equal-time events across sources, event_id, accumulated time_delta, t beyond end,
# times before start, unsorted and duplicate times within a source)
def realdata_worlds():
    rs = np.random.RandomState(2024)
    w1 = dict(src_id=1, end_time=100.0, s=1.0, q=1.0, sink_ids=[1, 2, 3],
              other_sources=[("RealData", {"src_id": 2, "times": [0.0, 0.5, 1.0, 3.0, 3.0, 7.25, 9.0,
                                                                 100.0]}),
                             ("RealData", {"src_id": 3, "times": [0.5, 2.0, 2.5, 8.0, 7.0, -1.0,
                                                                 101.0]})],
              edge_list=[(1, 1), (1, 3), (2, 1), (2, 2), (2, 3), (3, 3)])
    c1 = [0.0, 0.5, 2.0, 2.0, 7.25, 50.0, 99.0, 100.0, 120.0]
    sinks = list(range(1, 16))
    srcs = [3, 7, 12, 20]
    edges = []
    for sid in [10] + srcs:
        for y in rs.choice(sinks, rs.randint(2, 9), replace=False):
            edges.append((sid, int(y)))
    edges.append((99, 4))   # a source with one edge and times only past end_time
    others = [("RealData", {"src_id": sid, "times": list(np.round(rs.uniform(-2, 44, rs.randint(5, 30)) * 2) / 2)})
              for sid in srcs] + [("RealData", {"src_id": 99, "times": [41.0, 45.0]})]
    w2 = dict(src_id=10, end_time=40.0, s=1.0, q=1.0, sink_ids=sinks, other_sources=others,
              edge_list=edges)
    c2 = list(np.round(rs.uniform(0, 42, 25) * 2) / 2) + [0.0]
    # tiny times first: the accumulated State.time rounds (t_k > 2 time_{k-1})
    w3 = dict(src_id=4, end_time=3.0, s=1.0, q=1.0, sink_ids=[1, 2],
              other_sources=[("RealData", {"src_id": 2, "times": [1e-9, 3e-9, 0.1, 0.1 + 1e-12, 1.7,
                                                                 2.9999999]}),
                             ("RealData", {"src_id": 7, "times": [0.3, 1.0 / 3.0, 2.0 / 3.0, 3.0]})],
              edge_list=[(2, 1), (7, 1), (7, 2), (4, 2)])
    c3 = [1e-300, 0.1 + 1e-12, 0.7, 1.7]
    # multigraphs (duplicate edges, which Manager.__init__ accepts, opt_model.py:169-175):
    # every duplicated (source, sink) edge repeats that sink's rows of each event
    # (opt_model.py:306-307), so the pivot cells average consecutive ranks (k + 1/2, ...)
    # and carry them by ffill; also duplicated controlled edges and equal times
    w4 = dict(src_id=1, end_time=30.0, s=1.0, q=1.0, sink_ids=[1, 2, 3, 4],
              other_sources=[("RealData", {"src_id": 2, "times": [0.5, 1.0, 3.0, 3.0, 7.5, 12.0,
                                                                 20.0, 29.0]}),
                             ("RealData", {"src_id": 3, "times": [1.0, 2.0, 7.5, 8.0, 15.0, 25.0]}),
                             ("RealData", {"src_id": 5, "times": [4.0, 16.0, 16.0, 26.5]})],
              edge_list=[(1, 1), (1, 2), (1, 1), (2, 1), (2, 2), (2, 1), (2, 1), (3, 3), (3, 2),
                         (3, 3), (5, 4), (5, 1), (5, 4), (5, 4), (1, 4)])
    c4 = [0.0, 1.0, 5.0, 7.5, 14.0, 16.0, 22.0]
    edges5 = []
    rs5 = np.random.RandomState(77)
    for sid in (10, 11, 12, 13, 14):
        for y in rs5.choice(range(1, 9), 12, replace=True):   # random multiplicities
            edges5.append((sid, int(y)))
    w5 = dict(src_id=10, end_time=50.0, s=1.0, q=1.0, sink_ids=list(range(1, 9)),
              other_sources=[("RealData", {"src_id": sid,
                                           "times": list(np.round(rs5.uniform(0, 50, 20) * 4) / 4)})
                             for sid in (11, 12, 13, 14)],
              edge_list=edges5)
    c5 = list(np.round(rs5.uniform(0, 50, 15) * 4) / 4)
    return [("rd1", w1, c1, None), ("rd2", w2, c2, None), ("rd2m", w2, c2, 17), ("rd3", w3, c3, None),
            ("rdmg1", w4, c4, None), ("rdmg2", w5, c5, None), ("rdmg2m", w5, c5, 23)]


class BurstyMixin:
    """A static plugin broadcaster (the SimOpts.registerSource contract,
    opt_model.py:323-378, :768-771): N ~ Poisson(rate * T) burst centres, each with
    `size` posts at centre + Exp(0.05), rounded to 1e-3 (so different sources post
    at equal times).  Only numpy RandomState draws through self.random_state."""

    def __init__(self, src_id, seed, rate=0.2, size=3):
        super().__init__(src_id, seed)
        self.rate, self.size = rate, size
        self.is_dynamic = False
        self.times = None

    def initialize(self):
        T = self.end_time - self.start_time
        n = self.random_state.poisson(self.rate * T)
        c = self.random_state.uniform(self.start_time, self.end_time, n)
        off = self.random_state.exponential(0.05, (n, self.size))
        self.times = np.round((c[:, None] + off).ravel(), 3)

    def get_all_times(self):
        return self.times


def plugin_world():
    """Two Bursty sources + a RealData controlled source (create_manager_with_times):
    deterministic for given seeds; randomize_other_sources(u) reseeds the plugins."""
    w = dict(src_id=4, end_time=30.0, s=1.0, q=1.0, sink_ids=[1, 2, 3, 4, 5, 6],
             other_sources=[("Bursty", {"src_id": 2, "seed": 11, "rate": 0.3, "size": 3}),
                            ("Bursty", {"src_id": 6, "seed": 12, "rate": 0.2, "size": 4})],
             edge_list=[(2, 1), (2, 2), (2, 5), (6, 2), (6, 3), (6, 6), (4, 1), (4, 3), (4, 4),
                        (4, 6)])
    ctrl = [0.0, 1.5, 4.0, 9.25, 12.0, 20.0, 27.5]
    return w, ctrl, list(range(16))


class RenewalMixin:
    """A DYNAMIC plugin broadcaster (get_next_interval queried on every event,
    opt_model.py:351-369) that is self-driven: on its own events (and at the start) it
    draws a gamma(2, scale) gap through self.random_state; on every other source's event
    it returns None (the schedule stays)."""

    def __init__(self, src_id, seed, scale=0.6):
        super().__init__(src_id, seed)
        self.scale = scale

    def get_next_interval(self, event):
        if event is None or event.src_id == self.src_id:
            return self.random_state.gamma(2.0, self.scale)
        return None


class KnockedOffMixin:
    """A DYNAMIC plugin whose schedule reacts to other sources' events (the reference's
    SmartPoisson idea, opt_model.py:436-455): after its own post it waits; when another
    source's event knocks it off its followers' top it schedules a post Exp(rate) later."""

    def __init__(self, src_id, seed, rate=1.0):
        super().__init__(src_id, seed)
        self.rate = rate
        self.on_top = False

    def get_next_interval(self, event):
        if event is None:
            return self.random_state.exponential(scale=1.0 / self.rate)
        if event.src_id == self.src_id:
            self.on_top = True
            return float("inf")
        if self.on_top and set(event.sink_ids) & set(self.sink_ids):
            self.on_top = False
            return (self.get_current_time(event) - self.last_self_event_time +
                    self.random_state.exponential(scale=1.0 / self.rate))
        return None


def dyn_plugin_world():
    """A self-driven dynamic plugin (Renewal, src 2) + a static one (Bursty, src 6) + a
    RealData controlled source: deterministic for given seeds."""
    w = dict(src_id=4, end_time=30.0, s=1.0, q=1.0, sink_ids=[1, 2, 3, 4, 5, 6],
             other_sources=[("Renewal", {"src_id": 2, "seed": 21, "scale": 0.6}),
                            ("Bursty", {"src_id": 6, "seed": 12, "rate": 0.2, "size": 4})],
             edge_list=[(2, 1), (2, 2), (2, 5), (6, 2), (6, 3), (6, 6), (4, 1), (4, 3), (4, 4),
                        (4, 6)])
    ctrl = [0.0, 1.5, 4.0, 9.25, 12.0, 20.0, 27.5]
    return w, ctrl, list(range(16))


class GridBurstyMixin(BurstyMixin):
    """Bursty on the 0.25 grid: burst posts rounded to quarters (exact in binary), so
    its posts meet the other grid sources' times and each other's exactly."""

    def initialize(self):
        super().initialize()
        self.times = np.round(self.times * 4.0) / 4.0


class GridKnockMixin(KnockedOffMixin):
    """KnockedOff on the 0.5 grid: when another source's event knocks it off its
    followers' top it schedules its next post at the first half-integer at least
    Exp(rate) later.  With every other source on the 0.25 grid, every time and every
    difference run_dynamic forms is exact in binary, so its posts meet the static
    sources' times EXACTLY: the equal-time order of a dynamic source against static ones
    (opt_model.py:279-290) is exercised, not an ulp-level accident."""

    def get_next_interval(self, event):
        if event is None:
            return 0.5 * np.ceil(2.0 * self.random_state.exponential(scale=1.0 / self.rate))
        if event.src_id == self.src_id:
            self.on_top = True
            return float("inf")
        if self.on_top and set(event.sink_ids) & set(self.sink_ids):
            self.on_top = False
            t = 0.5 * np.ceil(2.0 * (self.get_current_time(event) +
                                     self.random_state.exponential(scale=1.0 / self.rate)))
            return t - self.last_self_event_time
        return None


def grid_tie_world():
    """A reactive dynamic plugin (GridKnock, src 7: the LARGEST src_id) beside a static
    plugin (GridBursty, src 6) and a RealData controlled source (src 4), all on binary
    grids: at an equal time the dynamic plugin plays first although its src_id is the
    largest (run_dynamic plays a static time only when strictly earlier)."""
    w = dict(src_id=4, end_time=30.0, s=1.0, q=1.0, sink_ids=[1, 2, 3, 4, 5, 6],
             other_sources=[("GridBursty", {"src_id": 6, "seed": 12, "rate": 0.3, "size": 3}),
                            ("GridKnock", {"src_id": 7, "seed": 21, "rate": 1.0})],
             edge_list=[(7, 1), (7, 2), (7, 5), (6, 2), (6, 3), (6, 6), (4, 1), (4, 3), (4, 4),
                        (4, 6)])
    ctrl = [0.0, 1.5, 2.5, 4.0, 5.5, 7.0, 9.25, 12.0, 13.5, 16.0, 20.0, 22.5, 25.0, 27.5]
    return w, ctrl, list(range(32))
