"""TEST INFRASTRUCTURE ONLY: CPU restatement oracle of the reference AIR path.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
only — never by the product package."""
