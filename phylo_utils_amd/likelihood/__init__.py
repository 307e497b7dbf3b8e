"""Likelihood engines: ``hip_likelihood_engine`` is the drop-in for the reference's
``phylo_utils.likelihood.numba_likelihood_engine`` (clv, lnl_node)."""
