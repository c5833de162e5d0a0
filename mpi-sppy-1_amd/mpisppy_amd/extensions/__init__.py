"""Extensions used by the spokes (xhatbase)."""
