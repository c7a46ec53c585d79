"""ba_amd -- MI355X-native batched OM(m) Byzantine-agreement engine.

Host side of libba_hip.so: the ctypes binding (lib), the ba.py-style general /
cluster objects (generals) and the REPL front end (repl).  The arithmetic lives
in the HIP kernels of ../csrc; nothing here computes a decision on the CPU.
"""
from .lib import (ATTACK, ENGINE_AUTO, ENGINE_FUSED, ENGINE_LEVELS, FAULTY_EXACT,  # noqa: F401
                  FAULTY_GIVEN, FAULTY_RANDOM, LIE_PHILOX, LIE_TABLE, ORDER_CONST,
                  ORDER_GIVEN, ORDER_RANDOM, OTHER, RETREAT, UNDEFINED, BAError, Engine,
                  MT, RunResult, load)

__all__ = ["Engine", "RunResult", "BAError", "load", "MT"]
