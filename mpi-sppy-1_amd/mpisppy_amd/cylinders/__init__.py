"""Hub / spoke cylinders (mirrors mpisppy/cylinders)."""
