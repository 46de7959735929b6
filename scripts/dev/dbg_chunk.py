"""Debug: chunked replay internals for one random df (workspace RpInfo + counts)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.test_gpu_replay_chunked import _random_df  # noqa: E402
from redqueen_amd import _lib as L  # noqa: E402

os.environ["RQ_RP_CHUNK"] = "1"
for n_events, n_sinks in ((2500, 4000), (3000, 1500), (2500, 3000), (2500, 3500)):
    rs = np.random.RandomState(n_events + n_sinks)
    sinks = np.unique(rs.randint(-10 ** 12, 10 ** 12, n_sinks + 50, dtype=np.int64))[:n_sinks]
    df = _random_df(rs, n_events, sinks, 0.0, 0.1, 0.2)
    n = len(df)
    lib = L.lib()
    Ks = np.asarray([1, 2], dtype=np.int32)
    for flags in (L.REPLAY_CHUNKED, L.REPLAY_CHUNKED | L.REPLAY_LARGE):
        nb = C.c_size_t()
        lib.rq_replay_workspace_size(n, 1, 2, flags, C.byref(nb))
        ws = torch.zeros(nb.value, dtype=torch.uint8, device="cuda")
        dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).cuda()  # noqa: E731
        t, s, k, e = dev(df.t.values, np.float64), dev(df.src_id.values, np.int64), dev(df.sink_id.values, np.int64), dev(df.event_id.values, np.int64)
        out = torch.empty(4, dtype=torch.float64, device="cuda")
        cnt = torch.empty(4, dtype=torch.int64, device="cuda")
        rc = lib.rq_metrics_replay(t.data_ptr(), s.data_ptr(), k.data_ptr(), e.data_ptr(), n, 1, float(df.t.max()) + 0.5,
                                   Ks.ctypes.data_as(L._pi32), 2, out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), None)
        torch.cuda.synchronize()
        info = ws[:32].cpu().numpy().view(np.int64)
        print(n_sinks, "flags", flags, "rc", rc, "rows", n, "uniq", df.sink_id.nunique(), "info n_piv/own/world", info[:3],
              "S,flags", ws[24:32].cpu().numpy().view(np.int32), "out", out.cpu().numpy(), "cnt", cnt.cpu().numpy(), flush=True)
