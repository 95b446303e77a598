"""Config object read by ``Generator`` (env.py:5-8 of the reference): a dict with attribute access."""


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self
