"""pettingzoo.ParallelEnv base-class stub (fixture generation only)."""


class ParallelEnv:
    metadata = {}
