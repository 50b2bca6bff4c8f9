"""StateLoader / StatePersister / InMemoryStateProvider (reference: analyzers/StateProvider.scala:
36-69).  States are the analyzers' own state objects (device frequency tables included)."""
from __future__ import annotations

import threading


class StateLoader:
    def load(self, analyzer):
        raise NotImplementedError


class StatePersister:
    def persist(self, analyzer, state) -> None:
        raise NotImplementedError


class InMemoryStateProvider(StateLoader, StatePersister):
    def __init__(self):
        self._states = {}
        self._lock = threading.Lock()

    def load(self, analyzer):
        with self._lock:
            return self._states.get(analyzer)

    def persist(self, analyzer, state) -> None:
        with self._lock:
            self._states[analyzer] = state

    def __str__(self):
        return "".join(f"{a} => {s}\n" for a, s in self._states.items())
