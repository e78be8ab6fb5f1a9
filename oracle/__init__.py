"""CPU restatement of the HyGrid hot path (test infrastructure only)."""
