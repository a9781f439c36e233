"""EpochCounter: iterable over epochs 1..limit, checkpointable (SpeechBrain semantics).

Its checkpoint file is SpeechBrain's: the current epoch as plain text; recovering from a
checkpoint that was not written at the end of an epoch replays that epoch (current - 1)."""


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

    # SpeechBrain's saver / recoverer pair for this object (plain-text file)
    def ckpt_save(self, path):
        with open(path, "w") as f:
            f.write(str(self.current))

    def ckpt_recover(self, path, end_of_epoch=True):
        with open(path) as f:
            saved = int(f.read().strip())
        self.current = saved if end_of_epoch else saved - 1
