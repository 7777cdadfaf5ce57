"""Serving: KServe-compatible model server, predictors, FT/Triton endpoint, SD service."""
