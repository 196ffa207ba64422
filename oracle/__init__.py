"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A CPU fp32 PyTorch restatement of the reference's SSL step (taindp98/Endoscopy-Image-Classification):
  * ViT forward in the timm-0.5.4 layout with the block arithmetic of code/models/conformer.py:8-72,
  * PolyLoss / consistency_loss of code/loss.py:103-164,308-364,
  * ModelEMA.update of code/ema.py:51-59,
  * one FixMatch step of code/fixmatch.py:91-131 (torch.optim.Adam, wd=0, code/optimizer.py:50-51).

It is PINNED against golden fixtures produced by running the reference itself in the build
container (tests/golden/make_golden.py, tests/test_oracle_golden.py).  It is imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker / the timed
CPU baseline -- never by the product package (endossl), which has no CPU fallback.
"""
