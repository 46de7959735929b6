"""redqueen_amd -- MI355X-native Monte-Carlo engine for RedQueen smart broadcasting.

Drop-in surface of the reference (MPI-SWS/RedQueen):
    from redqueen_amd.opt_model import SimOpts          # opt_model.py:755
    from redqueen_amd import utils as U                 # utils.py:84-176
    m = sim_opts.create_manager_with_opt(seed); m.run_dynamic()
    df = m.state.get_dataframe(); U.time_in_top_k(df, K=1, sim_opts=sim_opts)
plus the batched grid API in redqueen_amd.batch.  All simulation and metric
arithmetic runs in librq.so (gfx950 HIP kernels, include/rq.h).
"""
__version__ = "0.1.0"
