"""CPU oracle (test infrastructure only; see p2p_oracle.py header)."""
