class ComplexTensor:  # placeholder type, never instantiated on the ASR path
    pass
