"""dcrecommend on MI355X: the reference's package surface (dcrecommend.nn.DCUE, dcrecommend.dcue,
dcrecommend.datasets, dcrecommend.optim) over the HIP C ABI in include/dcue.h."""
