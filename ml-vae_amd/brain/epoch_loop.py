"""EpochCounter: iterable over epochs 1..limit, checkpointable (SpeechBrain semantics)."""


class EpochCounter:
    def __init__(self, limit):
        self.current = 0
        self.limit = int(limit)

    def __iter__(self):
        return self

    def __next__(self):
        if self.current < self.limit:
            self.current += 1
            return self.current
        raise StopIteration

    def state_dict(self):
        return {"current": self.current}

    def load_state_dict(self, sd):
        self.current = int(sd["current"])
