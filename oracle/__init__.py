"""Parity oracle for the CT-CLIP contrastive step — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package never imports anything from here.
"""
from . import ctclip_oracle, weights  # noqa: F401
