"""CPU oracle (TEST INFRASTRUCTURE ONLY): restatements of the reference's BitLinear hot path
and model used as the parity checker by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Never imported by the product package. See quant_oracle.py for how the
oracle is pinned (hand-derived KATs; the reference has no golden vectors and running it
here was denied)."""
