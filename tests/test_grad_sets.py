from akka_allreduce_1_amd.models.grad_sets import gradient_shapes, numel


def test_resnet50_parameter_count():
    shapes = gradient_shapes("resnet50")
    assert sum(numel(s) for _, s in shapes) == 25_557_032
    assert len(shapes) == 161


def test_llama3_8b_parameter_count():
    shapes = gradient_shapes("llama3_8b")
    total = sum(numel(s) for _, s in shapes)
    assert total == 8_030_261_248
    assert abs(total * 2 / 1e9 - 16.06) < 0.01
