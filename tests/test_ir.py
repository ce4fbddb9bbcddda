"""``internal/types/ir_test.go``, one test per Go subtest, each comparing
the whole object as the Go test does (``cmp.Equal`` / ``reflect.DeepEqual``,
``tests/goequal.py``).  ``tests/reference_ledger.json`` maps every Go subtest
to its test here."""

from goequal import assert_deep_equal

from move2kube_amd.models import collection
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes

DF = plantypes.NEW_DOCKERFILE


def C(name="name1", new=True):
    return irtypes.new_container(DF, name, new)


def new_ir():
    return irtypes.new_ir(plantypes.new_plan())


# -- TestAddVolume -------------------------------------------------------------

def test_add_volume_to_an_empty_service():
    v = {"name": "name1"}
    s = irtypes.Service()
    want = irtypes.Service()
    want.volumes = [v]
    s.add_volume(v)
    assert_deep_equal(s, want)


def test_add_volume_with_same_name_to_a_filled_service():
    v = {"name": "name1"}
    s = irtypes.Service()
    s.volumes = [v]
    want = irtypes.Service()
    want.volumes = [v]
    s.add_volume(v)
    assert_deep_equal(s, want)


# -- TestNewContainer ------------------------------------------------------------

def test_new_container():
    c = irtypes.new_container(DF, "name1", True)
    assert c.image_names == ["name1"] and c.new is True and c.new_files == {}
    want = irtypes.Container()
    want.container_build_type, want.image_names, want.new = DF, ["name1"], True
    assert_deep_equal(c, want)


# -- TestNewContainerFromImageInfo ---------------------------------------------

def test_new_container_from_image_with_tags():
    info = collection.ImageInfo()
    info.tags = ["tag1"]
    c = irtypes.new_container_from_image_info(info)
    assert_deep_equal(c.image_names, info.tags)
    assert_deep_equal(c.exposed_ports, info.ports)
    assert c.user_id == info.user_id
    assert_deep_equal(c.accessed_dirs, info.accessed_dirs)


def test_new_container_from_image_without_tags():
    info = collection.ImageInfo()
    c = irtypes.new_container_from_image_info(info)
    assert_deep_equal(c.image_names, info.tags)
    assert_deep_equal(c.exposed_ports, info.ports)
    assert c.user_id == info.user_id
    assert_deep_equal(c.accessed_dirs, info.accessed_dirs)


# -- TestContainerMerge ------------------------------------------------------------

def test_container_merge_2_empty_containers():
    c1, c2 = C("name1"), C("name2")
    want = C("name1")
    assert not c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_containers_that_share_no_image_names():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c2 = C("name2")
    c2.image_names = ["imgname4", "imgname5", "imgname6"]
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3"]
    assert not c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_containers_that_share_some_image_names():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c2 = C("name2", new=False)
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_2_new_containers_with_the_same_build_scripts():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c1.new_files["path1"] = "contents1"
    c2 = C("name2")
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    c2.new_files["path1"] = "contents1"
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    want.new_files["path1"] = "contents1"
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_2_new_containers_with_different_build_scripts():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c1.new_files["path1"] = "contents1"
    c2 = C("name2")
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    c2.new_files["path2"] = "contents2"
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    want.new_files["path1"] = "contents1"
    want.new_files["path2"] = "contents2"
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_2_new_containers_with_different_build_scripts_for_the_same_key():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c1.new_files["path1"] = "contents1"
    c2 = C("name2")
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    c2.new_files["path1"] = "contents2"
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    want.new_files["path1"] = "contents1"
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_2_new_containers_with_different_user_ids():
    c1 = C("name1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c1.user_id = 1
    c2 = C("name2")
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    c2.user_id = 2
    want = C("name1")
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    want.user_id = 1
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


def test_container_merge_new_into_old_with_different_user_ids_and_build_scripts():
    c1 = C("name1", new=False)
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    c1.user_id = 1
    c1.new_files["path1"] = "contents1"
    c2 = C("name2")
    c2.image_names = ["imgname3", "imgname4", "imgname5"]
    c2.user_id = 2
    c2.new_files["path2"] = "contents2"
    want = C("name1", new=False)
    want.image_names = ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]
    want.user_id = 2
    want.new_files["path2"] = "contents2"
    assert c1.merge(c2)
    assert_deep_equal(c1, want)


# -- TestAddFile -------------------------------------------------------------------

def test_add_file_new_script_to_an_empty_container():
    c = C()
    want = C()
    want.new_files["path1/foo/bar"] = "contents1"
    c.add_file("path1/foo/bar", "contents1")
    assert_deep_equal(c, want)


def test_add_file_same_script_at_the_same_path():
    c = C()
    c.new_files["path1/foo/bar"] = "contents1"
    want = C()
    want.new_files["path1/foo/bar"] = "contents1"
    c.add_file("path1/foo/bar", "contents1")
    assert_deep_equal(c, want)


def test_add_file_different_script_at_the_same_path():
    c = C()
    c.new_files["path1/foo/bar"] = "contents1"
    want = C()
    want.new_files["path1/foo/bar"] = "contents1"
    c.add_file("path1/foo/bar", "contents2")
    assert_deep_equal(c, want)


# -- TestAddExposedPort / TestAddImageName / TestAddAccessedDirs ---------------

def test_add_exposed_port_to_an_empty_container():
    c, want = C(), C()
    want.exposed_ports.append(8080)
    c.add_exposed_port(8080)
    assert_deep_equal(c, want)


def test_add_already_exposed_port_to_a_filled_container():
    c, want = C(), C()
    c.exposed_ports.append(8080)
    want.exposed_ports.append(8080)
    c.add_exposed_port(8080)
    assert_deep_equal(c, want)


def test_add_image_name_to_an_empty_container():
    c, want = C(), C()
    want.image_names.append("img1")
    c.add_image_name("img1")
    assert_deep_equal(c, want)


def test_add_existing_image_name_to_a_filled_container():
    c, want = C(), C()
    c.image_names.append("img1")
    want.image_names.append("img1")
    c.add_image_name("img1")
    assert_deep_equal(c, want)


def test_add_accessed_dir_to_an_empty_container():
    c, want = C(), C()
    want.accessed_dirs.append("dir1")
    c.add_accessed_dirs("dir1")
    assert_deep_equal(c, want)


def test_add_existing_accessed_dir_to_a_filled_container():
    c, want = C(), C()
    c.accessed_dirs.append("dir1")
    want.accessed_dirs.append("dir1")
    c.add_accessed_dirs("dir1")
    assert_deep_equal(c, want)


# -- TestNewIR / TestIRMerge -------------------------------------------------------

def test_new_ir():
    ir = new_ir()
    assert ir.containers == [] and ir.services == {} and ir.storages == [] and ir.values.global_variables == {}
    assert_deep_equal(ir, new_ir())


def test_ir_merge_2_empty_irs():
    ir1, ir2, want = new_ir(), new_ir(), new_ir()
    ir1.merge(ir2)
    assert_deep_equal(ir1, want)


def test_ir_merge_2_irs_with_different_names():
    ir1, ir2, want = new_ir(), new_ir(), new_ir()
    ir1.name, ir2.name, want.name = "name1", "name2", "name1"
    ir1.merge(ir2)
    assert_deep_equal(ir1, want)


def test_ir_merge_an_ir_with_a_name_into_an_ir_with_an_empty_name():
    ir1, ir2, want = new_ir(), new_ir(), new_ir()
    ir1.name, ir2.name, want.name = "", "name1", "name1"
    ir1.merge(ir2)
    assert_deep_equal(ir1, want)


def test_ir_merge_2_filled_irs():
    c1 = C("contname1")
    c1.image_names = ["imgname1", "imgname2", "imgname3"]
    s1 = irtypes.Storage(name="storage1")
    svc1 = irtypes.Service("svcname1")
    svc1.replicas = 2
    svc2 = irtypes.Service("svcname1")
    svc2.replicas = 4
    ir1 = new_ir()
    ir1.services["svcname1"] = svc1
    ir2 = new_ir()
    ir2.services["svcname1"] = svc2
    ir2.containers.append(c1)
    ir2.storages.append(s1)
    want = new_ir()
    want.services["svcname1"] = svc2
    want.containers.append(c1)
    want.storages.append(s1)
    ir1.merge(ir2)
    assert_deep_equal(ir1, want)


# -- TestStorageMerge ----------------------------------------------------------------

def test_storage_merge_empty_into_empty():
    s1, s2, want = irtypes.Storage(), irtypes.Storage(), irtypes.Storage()
    assert s1.merge(s2)
    assert_deep_equal(s1, want)


def test_storage_merge_storages_with_different_names():
    s1, s2, want = irtypes.Storage(name="name1"), irtypes.Storage(name="name2"), irtypes.Storage(name="name1")
    assert not s1.merge(s2)
    assert_deep_equal(s1, want)


def test_storage_merge_filled_into_filled():
    s1 = irtypes.Storage(content={"key1": b"val1"})
    s2 = irtypes.Storage(content={"key2": b"val2"})
    want = irtypes.Storage(content={"key2": b"val2"})
    assert s1.merge(s2)
    assert_deep_equal(s1, want)


# -- TestAddContainer / TestAddStorage ------------------------------------------

def test_add_container_to_an_empty_ir():
    c = C()
    ir, want = new_ir(), new_ir()
    want.containers.append(c)
    ir.add_container(c)
    assert_deep_equal(ir, want)


def test_add_existing_container_to_a_filled_ir():
    c1 = C()
    ir, want = new_ir(), new_ir()
    ir.containers.append(c1)
    want.containers.append(C())
    ir.add_container(c1)
    assert_deep_equal(ir, want)


def test_add_storage_to_an_empty_ir():
    s = irtypes.Storage()
    ir, want = new_ir(), new_ir()
    want.storages.append(s)
    ir.add_storage(s)
    assert_deep_equal(ir, want)


def test_add_existing_storage_to_a_filled_ir():
    s = irtypes.Storage()
    ir, want = new_ir(), new_ir()
    ir.storages.append(s)
    want.storages.append(s)
    ir.add_storage(s)
    assert_deep_equal(ir, want)


# -- TestGetContainer --------------------------------------------------------------

def test_get_container_non_existent_image_name_from_empty_ir():
    assert new_ir().get_container("imgname1")[1] is False


def test_get_container_non_existent_image_name_from_filled_ir():
    ir = new_ir()
    ir.containers.append(C("contname1"))
    assert ir.get_container("imgname1")[1] is False


def test_get_container_image_name_from_filled_ir():
    c1 = C("contname1")
    c1.image_names.append("imgname1")
    ir = new_ir()
    ir.containers.append(c1)
    got, ok = ir.get_container("imgname1")
    assert ok and got is c1


def test_get_container_image_url_from_filled_ir():
    c1 = C("contname1")
    c1.image_names.append("imgname1")
    ir = new_ir()
    ir.containers.append(c1)
    ir.kubernetes.registry_url = "registry1.com"
    got, ok = ir.get_container("registry1.com/namespace/imgname1")
    assert ok and got is c1
