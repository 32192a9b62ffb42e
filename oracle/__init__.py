"""Parity oracle (CPU restatement of the reference) — test infrastructure only; see nconv_ref.py."""
