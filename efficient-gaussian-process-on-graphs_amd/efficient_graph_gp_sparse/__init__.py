"""Drop-in mirror of the reference's sparse package ``efficient_graph_gp_sparse`` on the MI355X engine."""
