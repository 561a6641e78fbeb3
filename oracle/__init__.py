"""CPU oracle — test infrastructure only (see rsa_oracle.py header)."""
