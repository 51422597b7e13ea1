"""PyTorch surface mirroring the reference's ``kungfu.torch`` package
(srcs/python/kungfu/torch/{ops,optimizers}): same names, arguments and
meaning, with the reduction on the MI355X bucket path."""
