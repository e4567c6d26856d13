"""Drop-in mirror of the reference's dense package ``efficient_graph_gp`` on the MI355X engine.

Module paths and signatures follow the reference; every computation runs in
``grf_amd`` (HIP kernels).  Extra keyword-only arguments: ``rng`` ("reference" =
bit-faithful PCG64 replay, "philox" = fast counter RNG) and ``device``.
"""
