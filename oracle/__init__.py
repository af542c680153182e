"""CPU restatement of the reference block codec -- test infrastructure only (see lsmblk_oracle.c)."""
