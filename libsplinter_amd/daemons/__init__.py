"""Long-running sidecars (splinference-compatible embedder, completion demo)."""
