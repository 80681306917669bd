"""bench.py host logic (no GPU): workload shapes match SURVEY.md §8 configs."""
import bench


def test_yolov8n_backbone_matches_survey_c4():
    layers = bench.yolov8n_backbone()
    assert len(layers) == 27
    assert sum(co * h * h for _, co, _, _, h in layers) == 2_137_600      # act elem / image
    assert sum(ci * co * k * k for ci, co, k, _, _ in layers) == 1_267_632   # weight elems
    assert layers[0] == (3, 16, 3, 2, 160) and layers[-1] == (512, 256, 1, 1, 10)
