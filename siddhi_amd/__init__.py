"""siddhi_amd — MI355X-native batch NFA matcher for Siddhi's pattern/sequence engine.

The product is libsiddhi_hip.so (C-ABI, include/siddhi_hip.h); this package is its
host-side mirror of the SiddhiManager / SiddhiAppRuntime / InputHandler /
StreamCallback API plus the SiddhiQL subset compiler that lowers apps to the
boundary descriptor (include/sh_query.h).
"""
from .runtime import (Event, InMemoryPersistenceStore, InputHandler, NoPersistenceStoreException, QueryCallback,
                      SiddhiAppCreationException, SiddhiAppRuntime, SiddhiAppRuntimeException, SiddhiManager,
                      StreamCallback)

__all__ = ["SiddhiManager", "SiddhiAppRuntime", "InputHandler", "StreamCallback", "QueryCallback",
           "Event", "SiddhiAppCreationException", "SiddhiAppRuntimeException", "InMemoryPersistenceStore",
           "NoPersistenceStoreException"]
