"""Device action drivers (fair / FIFO / random) — see csrc/policy.h."""
