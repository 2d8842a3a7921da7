"""Model families served by the framework (Nomic-BERT embedder)."""
