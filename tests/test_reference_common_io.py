"""The typed-file constructors (``types/collection/*_test.go``,
``types/qaengine/cache_test.go``).  The file IO subtests of
``internal/common/utils_test.go`` are in ``test_reference_utils.py``."""

import pytest

from move2kube_amd.models import collection, qa
from move2kube_amd.utils import constants

pytestmark = pytest.mark.reference


@pytest.mark.parametrize("obj,kind", [
    pytest.param(collection.ImageInfo(), collection.IMAGE_METADATA_KIND, id="TestNewImageInfo"),
    pytest.param(collection.CfContainerizers(), collection.CF_CONTAINERIZERS_KIND, id="TestNewCfContainerizers"),
    pytest.param(collection.CfInstanceApps(), collection.CF_INSTANCE_APPS_KIND, id="TestNewCfInstanceApps"),
    pytest.param(qa.Cache("cache.yaml"), qa.QACACHE_KIND, id="TestNewCache"),
])
def test_new_typed_files(obj, kind):
    assert obj.kind == kind
    assert obj.api_version == constants.SCHEME_GROUP_VERSION == "move2kube.konveyor.io/v1alpha1"
    doc = obj.to_yaml()
    assert doc["kind"] == kind and doc["apiVersion"] == constants.SCHEME_GROUP_VERSION
