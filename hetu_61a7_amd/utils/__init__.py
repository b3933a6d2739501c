"""Auxiliary subsystems: checkpointing, timers/profilers, tracing, hipGraph."""
