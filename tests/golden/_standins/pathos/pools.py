# Fixture-generation stand-in for pathos.pools.ProcessPool: a stdlib fork pool
# with the same map() semantics. The generator only uses num_cores=1, so this
# is imported but not exercised.
import multiprocessing as _mp


class ProcessPool:
    def __init__(self, n=None):
        self._n = n

    def __enter__(self):
        self._p = _mp.get_context("fork").Pool(self._n)
        return self

    def __exit__(self, *exc):
        self._p.close()
        self._p.join()
        return False

    def map(self, f, xs):
        return self._p.map(f, list(xs))
