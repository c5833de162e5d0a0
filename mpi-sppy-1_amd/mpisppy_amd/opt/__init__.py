"""PH optimisers (mirrors mpisppy/opt)."""
