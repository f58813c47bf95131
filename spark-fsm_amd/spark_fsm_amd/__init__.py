"""spark_fsm_amd — MI355X engine for spark-fsm's hot path (SPADE + TSR).

The product is libfsm.so (C ABI in include/fsm.h); this package is the host
mirror of the reference's Scala API over it.
"""
from ._lib import (FsmError, FsmParseError, MODE_SPADE, MODE_TSR, LIB_PATH, FSM_OK, FSM_EINVAL,  # noqa: F401
                   FSM_EPARSE, FSM_EDEVICE, FSM_ENOMEM, FSM_ECOMM, FSM_ELIMIT)
from .engine import Engine, DB, default_engine  # noqa: F401
from .dist import comm_unique_id, shard_plan, TorchHostComm  # noqa: F401
from .api import (Pattern, Rule, extract_rdd_patterns, extract_rdd_rules,  # noqa: F401
                  spade_actor_patterns, tsr_actor_rules)
from .builder import TokenDB, ingest, build as spmf_build  # noqa: F401
from .results import PatternSet, RuleSet  # noqa: F401
