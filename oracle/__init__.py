"""CPU oracle — test infrastructure only (see oracle/bopx_oracle.c)."""
