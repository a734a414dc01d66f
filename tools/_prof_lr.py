import cProfile, pstats, sys, os, io
sys.path.insert(0, os.getcwd())
from tools import lr_he_demo as D
from xfl_amd.paillier import Paillier
key = Paillier.context(2048, djn_on=True)
D.run(epochs=1, key=key)
pr = cProfile.Profile()
pr.enable()
rec = D.run(epochs=2, key=key)
pr.disable()
print(rec["per_batch_ms"])
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue()[:6000])
