"""A/B helper: run ``bench.py`` with a no-op global optimizer step pre-hook registered, which
sends :meth:`xdot.FusedAdamW.step` down torch's wrapped path (profiler range + hook loops), the
pre-round-4 behaviour.  ``python benchmarks/micro/optim_hooked.py <bench.py args>``."""
import os
import runpy
import sys

from torch.optim.optimizer import register_optimizer_step_pre_hook

register_optimizer_step_pre_hook(lambda opt, args, kwargs: None)
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root)
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
