"""CPU oracle (test infrastructure only).  See kge_oracle.py."""
