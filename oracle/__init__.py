"""Test infrastructure: CPU oracle(s) for the decode path.  Never imported by ``adaptive_amd``."""
