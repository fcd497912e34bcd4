"""CPU ORACLE — test infrastructure only (see oracle/cpu_ref.py for the rules and the pinning)."""
