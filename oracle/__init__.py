"""CPU oracle — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg).
Never imported by the product package `bcnf_amd`."""
