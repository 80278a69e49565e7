"""ORACLE (test infrastructure only): CPU restatements of the reference path and the golden-fixture generator.
Only tests/, __graft_entry__.smoke() and bench.py (cpu_baseline) may import this package; the product never does."""
