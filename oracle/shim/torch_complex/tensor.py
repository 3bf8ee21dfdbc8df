"""TEST INFRASTRUCTURE stand-in for torch_complex.tensor.ComplexTensor (torch_complex is not
in this image; setup.py requires it unpinned): the (real, imag) pair and the members the
single-channel DefaultFrontend path uses (espnet2/asr/frontend/default.py:89-131: dim(),
.real, .imag).  Anything else is absent on purpose."""


class ComplexTensor:
    def __init__(self, real, imag=None):
        self.real = real
        self.imag = imag if imag is not None else real.new_zeros(real.shape)

    def dim(self):
        return self.real.dim()

    @property
    def shape(self):
        return self.real.shape

    def size(self, *args):
        return self.real.size(*args)
