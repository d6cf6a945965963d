"""Runtime utilities: communicators, flags, profiling, memory planning, consistency checks."""
