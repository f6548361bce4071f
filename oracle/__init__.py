"""CPU oracle for Doorman's lease algorithms — test infrastructure only (see doorman_oracle.h)."""
