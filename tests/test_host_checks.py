"""Host-side argument checks of the drop-in (CPU, no GPU needed)."""
import pytest
import torch


def test_class_label_range_check():
    """loss.check_class_labels mirrors torch.nn.functional.one_hot's errors on the
    reference's loss targets (loss.py:59-73) before any label reaches the native loss."""
    from graph_neural_network_for_radar_perception_amd.loss import check_class_labels
    ok = torch.tensor([0, 6, 3])
    check_class_labels([(ok, 7), (torch.tensor([0, 1]), 2), (torch.zeros(0, dtype=torch.int64), 7)])
    with pytest.raises(RuntimeError, match='smaller than num_classes'):
        check_class_labels([(ok, 7), (torch.tensor([0, 2]), 2)])
    with pytest.raises(RuntimeError, match='non-negative'):
        check_class_labels([(torch.tensor([-1, 0]), 7)])
    # the reference's own message for the same input
    with pytest.raises(RuntimeError, match='smaller than num_classes'):
        torch.nn.functional.one_hot(torch.tensor([0, 2]), 2)
