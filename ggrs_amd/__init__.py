"""ggrs_amd — MI355X-native batched rollback resimulation with GGRS semantics.

The hot path is the GGRS SyncTestSession resimulation (request stream
SaveGameState/LoadGameState/AdvanceFrame, /root/reference
src/sessions/sync_test_session.rs) executed for thousands of sessions per
HIP launch.  Public surface mirrors the reference: ``SessionBuilder``,
``SyncTestSession``, ``GGRSError`` and its variants, ``GGRSRequest``.
"""
from .session import (  # noqa: F401
    NULL_FRAME,
    DeviceError,
    Game,
    GGRSError,
    GGRSRequest,
    InputStatus,
    InvalidRequest,
    MismatchedChecksum,
    NotSynchronized,
    Panic,
    PredictionThreshold,
    RequestKind,
    SessionBuilder,
    SpectatorTooFarBehind,
    SyncTestSession,
    decode_ex_game,
)
from .synth import SEED, synth_inputs  # noqa: F401
from .p2p import P2PSession, PlayerType, synth_network  # noqa: F401

__version__ = "0.1.0"
