"""ORACLE -- test infrastructure only (CPU restatement of the reference's Groth16
hot path).  Importable only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  Never imported by bellman-mpc_amd/."""
