// Frontend contract tests of the JWA / VWA / TWA pages and the common-lib components, against the
// reference's Cypress fixtures (crud-web-apps/*/frontend/cypress/fixtures/*.json, read in place:
// argv[2] = the crud-web-apps directory) and the assertions of its Cypress specs:
//   jupyter/frontend/cypress/e2e/main-page.cy.ts  (name order, status icons, Namespace column)
//   jupyter/frontend/cypress/e2e/form-page.cy.ts  (workspace name / size / access mode from the
//                                                   config, data-volume mount follows its name
//                                                   until edited)
//   volumes/frontend/cypress/e2e/index-page.cy.ts, tensorboards/frontend/cypress/e2e/index-page.cy.ts
// No browser: the pages' pure parts render to strings and are checked here with node.
"use strict";
const assert = require("assert");
const fs = require("fs");
const path = require("path");

global.window = global;
global.document = { cookie: "" };
global.location = { search: "" };
global.localStorage = { getItem: () => null, setItem: () => {} };
global.addEventListener = () => {};
global.parent = global;

const WEB = path.join(__dirname, "../../kubeflow_rm_amd/webapps");
const kf = require(path.join(WEB, "crud_backend/static/kf.js"));
global.kf = kf;
const JWA = require(path.join(WEB, "jupyter/static/assets/app.js"));
const VWA = require(path.join(WEB, "volumes/static/assets/app.js"));
const TWA = require(path.join(WEB, "tensorboards/static/assets/app.js"));
const FIX = process.argv[2];
const fixture = (app, name) => JSON.parse(fs.readFileSync(path.join(FIX, app, "frontend/cypress/fixtures", name + ".json"), "utf8"));

const tests = [];
const test = (name, fn) => tests.push([name, fn]);

// cells of one column, in rendered row order
function column(html, title) {
  const re = new RegExp(`<td data-cy-resource-table-row="${title}">([\\s\\S]*?)</td>`, "g");
  const out = [];
  let m;
  while ((m = re.exec(html)) !== null) out.push(m[1]);
  return out;
}
function iconOf(cell) {
  if (cell.includes('data-icon="spinner"')) return "spinner";
  const m = cell.match(/data-icon="([^"]+)"/);
  return m ? m[1] : null;
}
const EXPECTED_ICON = { ready: "check_circle", stopped: "custom:stoppedResource", unavailable: "timelapse",
                        warning: "warning", waiting: "spinner", terminating: "spinner" };

function checkTable(rows, columns) {
  const html = kf.renderTable({ columns }, rows);
  // Table is sorted by Name in ascending order by default (the fixtures are sorted by name too)
  const names = column(html, "Name");
  assert.strictEqual(names.length, rows.length);
  names.forEach((cell, i) => assert.ok(cell.includes(kf.esc(rows[i].name)), `${cell} !~ ${rows[i].name}`));
  column(html, "Status").forEach((cell, i) => {
    const want = EXPECTED_ICON[rows[i].status.phase];
    if (want) assert.strictEqual(iconOf(cell), want, `${rows[i].name}: ${rows[i].status.phase}`);
  });
  return html;
}

test("JWA main page: every notebook name, in name order, with the reference status icons", () => {
  const nbs = fixture("jupyter", "notebooks").notebooks;
  const html = checkTable(nbs, JWA.columns(false));
  assert.ok(html.includes('data-cy-table-header-row="Name"'));
  assert.ok(!html.includes('data-cy-table-header-row="Namespace"'));
  // GPU / CPU / memory cells come straight from the backend row
  assert.deepStrictEqual(column(html, "CPUs"), nbs.map((n) => kf.esc(n.cpu)));
});

test("JWA main page: a Namespace column when showing all namespaces", () => {
  const nbs = fixture("jupyter", "notebooks").notebooks;
  const html = kf.renderTable({ columns: JWA.columns(true) }, nbs);
  assert.ok(html.includes('data-cy-table-header-row="Namespace"'));
  assert.deepStrictEqual(column(html, "Namespace"), nbs.map((n) => n.namespace));
  const merged = JWA.merge([[{ name: "b", namespace: "x" }], [{ name: "a", namespace: "y" }]]);
  assert.deepStrictEqual(kf.sortedRows({ columns: JWA.columns(true) }, merged).map((r) => r.name), ["a", "b"]);
});

test("JWA form: workspace volume name / size / access mode from the config", () => {
  const cfg = fixture("jupyter", "config").config;
  const f = JWA.formDefaults(cfg, "");
  assert.strictEqual(f.workspace.name, "-workspace");  // '{notebook-name}-workspace' with an empty name
  assert.strictEqual(f.workspace.size, "20");           // '20Gi'
  assert.strictEqual(f.workspace.accessMode, "ReadWriteMany");
  assert.strictEqual(JWA.formDefaults(cfg, "test").workspace.name, "test-workspace");
  assert.strictEqual(f.cpu, "0.5");
  assert.strictEqual(f.memory, "1.0Gi");
  assert.strictEqual(f.cpuLimit, "");                   // limitFactor "none"
  assert.strictEqual(f.shm, true);
});

test("JWA form: a data volume's mount follows its name until the mount is edited", () => {
  let v = JWA.newDataVolume("", 1);
  v = JWA.renameDataVolume(v, "new-volume-name");
  assert.strictEqual(v.mount, "/home/jovyan/new-volume-name");
  let d = JWA.editMount(JWA.newDataVolume("", 1), "dirty");
  d = JWA.renameDataVolume(d, "new-volume-name");
  assert.notStrictEqual(d.mount, "/home/jovyan/new-volume-name");
  assert.strictEqual(d.mount, "dirty");
});

test("JWA form: CPU / memory limits from the admin's limitFactor (form-cpu-ram)", () => {
  assert.strictEqual(JWA.limitFrom("1", "1.2", ""), "1.2");
  assert.strictEqual(JWA.limitFrom("2Gi", "1.2", "Gi"), "2.4Gi");
  assert.strictEqual(JWA.limitFrom("0.5", "none", ""), "");
  const cfg = JSON.parse(JSON.stringify(fixture("jupyter", "config").config));
  cfg.cpu.limitFactor = "1.2";
  cfg.memory.limitFactor = "1.2";
  const f = JWA.formDefaults(cfg, "nb");
  assert.strictEqual(f.cpuLimit, "0.6");
  assert.strictEqual(f.memoryLimit, "1.2Gi");
});

test("JWA form: request body and validation", () => {
  const cfg = fixture("jupyter", "config").config;
  const f = JWA.formDefaults(cfg, "my-nb");
  f.gpus = { num: "2", vendor: "amd.com/gpu" };
  f.cpuLimit = "1";
  f.datavols = [JWA.renameDataVolume(JWA.newDataVolume("my-nb", 1), "data1")];
  const b = JWA.buildBody(f, cfg, "team");
  assert.strictEqual(b.name, "my-nb");
  assert.strictEqual(b.namespace, "team");
  assert.deepStrictEqual(b.gpus, { num: "2", vendor: "amd.com/gpu" });
  assert.strictEqual(b.cpuLimit, "1");
  assert.ok(!("memoryLimit" in b));
  assert.deepStrictEqual(b.workspace.newPvc.spec, { resources: { requests: { storage: "20Gi" } }, accessModes: ["ReadWriteMany"] });
  assert.strictEqual(b.workspace.newPvc.metadata.name, "{notebook-name}-workspace");
  assert.strictEqual(b.datavols[0].mount, "/home/jovyan/data1");
  assert.strictEqual(b.datavols[0].newPvc.metadata.name, "data1");
  assert.deepStrictEqual(JWA.validate(f), []);
  const bad = Object.assign({}, f, { name: "Bad_Name", cpu: "abc", memory: "2Gi", memoryLimit: "1Gi" });
  const errs = JWA.validate(bad);
  assert.ok(errs.some((e) => e.includes("lowercase")), errs);
  assert.ok(errs.some((e) => e.includes("Invalid CPU")), errs);
  assert.ok(errs.some((e) => e.includes("Memory limit must be greater")), errs);
  // a readOnly config field is not sent (the backend answers 400 otherwise)
  const ro = JSON.parse(JSON.stringify(cfg));
  ro.shm.readOnly = true;
  ro.cpu.readOnly = true;
  const b2 = JWA.buildBody(f, ro, "team");
  assert.ok(!("shm" in b2) && !("cpu" in b2) && !("cpuLimit" in b2));
});

test("JWA form: Custom (Advanced) volumes edit the newPvc / existingSource as YAML (form-new/volume)", () => {
  const cfg = fixture("jupyter", "config").config;
  const f = JWA.formDefaults(cfg, "my-nb");
  // typeChanged(CUSTOM) dumps the current PVC into the editor
  f.workspace = JWA.toCustom(f.workspace);
  assert.strictEqual(f.workspace.yaml, kf.toYaml(JWA.volumeSpec(JWA.formDefaults(cfg, "my-nb").workspace)));
  assert.ok(f.workspace.yaml.includes("storage: 20Gi"), f.workspace.yaml);
  f.workspace = JWA.editCustom(f.workspace, f.workspace.yaml.replace("20Gi", "50Gi") + "\n  storageClassName: fast");
  const dv = JWA.toCustom(Object.assign(JWA.newDataVolume("my-nb", 1), { type: "existing", existing: "data" }));
  assert.deepStrictEqual(dv.spec, { persistentVolumeClaim: { claimName: "data" } });
  f.datavols = [JWA.editCustom(dv, "nfs:\n  server: 10.0.0.1\n  path: /exports")];
  let b = JWA.buildBody(f, cfg, "team");
  assert.strictEqual(b.workspace.newPvc.spec.resources.requests.storage, "50Gi");
  assert.strictEqual(b.workspace.newPvc.spec.storageClassName, "fast");
  assert.deepStrictEqual(b.datavols[0], { mount: dv.mount, existingSource: { nfs: { server: "10.0.0.1", path: "/exports" } } });
  assert.deepStrictEqual(JWA.validate(f), []);
  // a parse error keeps the last good spec and is reported; back to the plain form drops the YAML
  const broken = JWA.editCustom(f.datavols[0], "nfs:\n  server: a\n   path: b");
  assert.deepStrictEqual(broken.spec, f.datavols[0].spec);
  assert.ok(broken.yamlError.startsWith("bad indentation"), broken.yamlError);
  assert.ok(JWA.validate(Object.assign({}, f, { datavols: [broken] })).some((e) => e.startsWith("Data volume: bad indentation")));
  const plain = JWA.fromCustom(broken);
  b = JWA.buildBody(Object.assign({}, f, { datavols: [plain] }), cfg, "team");
  assert.deepStrictEqual(b.datavols[0].existingSource, { persistentVolumeClaim: { claimName: "data" } });
  assert.ok(JWA.kindOptions(plain).includes('value="pvc" selected') && JWA.kindOptions(dv).includes('value="custom" selected'));
});

test("JWA notebook page YAML tab: Notebook or Pod, with the component's placeholder texts", () => {
  const nb = { metadata: { name: "a" } }, pod = { metadata: { name: "a-0" } };
  assert.strictEqual(JWA.yamlTabText("notebook", nb), kf.toYaml(nb));
  assert.strictEqual(JWA.yamlTabText("notebook", null), "No data has been found...");
  assert.strictEqual(JWA.yamlTabText("pod", nb, null, false), "Pod information is still being loaded.");
  assert.strictEqual(JWA.yamlTabText("pod", nb, null, true), "No pod available for this notebook.");
  assert.strictEqual(JWA.yamlTabText("pod", nb, pod, true), kf.toYaml(pod));
});

test("JWA notebook overview: resources, type, volumes by kind, configurations, env groups (notebook-page/overview)", () => {
  const nb = {
    metadata: { name: "nb", namespace: "team", labels: { "access-ml-pipeline": "true", app: "nb" },
                annotations: { "notebooks.kubeflow.org/server-type": "group-one", "notebooks.kubeflow.org/creator": "user@x" } },
    spec: { template: { spec: {
      containers: [{ name: "sidecar" }, { name: "nb", image: "img:1", env: [{ name: "A", value: "1" }],
                     resources: { requests: { cpu: "500m", memory: "1Gi" }, limits: { cpu: "1" } } }],
      volumes: [{ name: "cm", configMap: { name: "c" } }, { name: "ws", persistentVolumeClaim: { claimName: "ws" } },
                { name: "dshm", emptyDir: { medium: "Memory" } }, { name: "tmp", emptyDir: {} }, { name: "s", secret: {} },
                { name: "data", persistentVolumeClaim: { claimName: "data" } }, { name: "x", nfs: {} }] } } },
  };
  const ov = JWA.overview(nb);
  assert.deepStrictEqual(ov, { notebookType: "VSCode", sharedMemory: "Yes", notebookCreator: "user@x", cpuRequests: "500m",
                               cpuLimits: "1", memoryRequests: "1Gi", memoryLimits: null, dockerImage: "img:1" });
  assert.strictEqual(JWA.overview({ metadata: { annotations: {} } }).notebookType, "empty");
  assert.strictEqual(JWA.overview({ metadata: {}, spec: { template: { spec: {} } } }).sharedMemory, "null");
  const g = JWA.volGroups(nb);
  assert.deepStrictEqual(g.map((x) => x.name), ["PersistentVolumeClaims", "ConfigMaps", "Memory-backed Volumes", "Ephemerals", "Secrets", "Other Volumes"]);
  assert.deepStrictEqual(g[0].items, [{ name: "ws", url: "/volumes/volume/details/team/ws" }, { name: "data", url: "/volumes/volume/details/team/data" }]);
  const pds = [
    { metadata: { name: "add-ml-pipeline" }, spec: { desc: "Allow access", selector: { matchLabels: { "access-ml-pipeline": "true" } },
      env: [{ name: "KF_PIPELINES_SA_TOKEN_PATH", value: "/var/run/secrets/token" }], volumes: [{ name: "tok" }] } },
    { metadata: { name: "other" }, spec: { selector: { matchLabels: { nope: "true" } }, env: [{ name: "B", value: "2" }] } },
  ];
  const cfgs = JWA.configurations(nb, pds);
  assert.deepStrictEqual(cfgs.map((c) => c.name), ["add-ml-pipeline"]);
  assert.ok(!JWA.configurationYaml(cfgs[0]).includes("name: add-ml-pipeline") && JWA.configurationYaml(cfgs[0]).includes("Description: Allow access"));
  assert.strictEqual(JWA.configurationYaml(null), "No information available about the configuration");
  assert.strictEqual(JWA.podDefaultsMessage(true, []), "No configurations available for this notebook.");
  assert.strictEqual(JWA.podDefaultsMessage(false, []), "");
  const pod = { metadata: { name: "nb-0", labels: { "notebook-name": "nb" } }, status: { podIP: "10.0.0.7" },
                spec: { containers: [{ name: "nb", env: [{ name: "A", value: "1" }, { name: "KF_PIPELINES_SA_TOKEN_PATH", value: "/var/run/secrets/token" },
                                                        { name: "IP", valueFrom: { fieldRef: { fieldPath: "status.podIP" } } }] }] } };
  assert.deepStrictEqual(JWA.envGroups(nb, pod, pds), [
    { name: "Notebook CR", chips: ["A: 1"] },
    { name: "add-ml-pipeline (Configuration)", chips: ["KF_PIPELINES_SA_TOKEN_PATH: /var/run/secrets/token"] },
    { name: "Other", chips: ["IP: 10.0.0.7"] }]);
  assert.deepStrictEqual(JWA.envGroups(nb, null, pds), [{ name: "Notebook CR", chips: ["A: 1"] }]);
});

test("JWA form storage class: default class leaves storageClassName out; an explicit or empty class is sent", () => {
  const v = JWA.newDataVolume("nb", 1);
  assert.ok(!("storageClassName" in JWA.volumeSpec(v).spec));
  assert.strictEqual(JWA.volumeSpec(Object.assign({}, v, { useDefaultSC: false, storageClass: "fast" })).spec.storageClassName, "fast");
  assert.strictEqual(JWA.volumeSpec(Object.assign({}, v, { useDefaultSC: false, storageClass: "" })).spec.storageClassName, "");
  const opts = JWA.storageClassOptions(["fast", "slow"], v, "slow");
  assert.ok(opts.startsWith('<option value="">Empty storage class</option>') && opts.includes('<option value="slow" selected>'), opts);
  const cfg = JSON.parse(JSON.stringify(fixture("jupyter", "config").config));
  assert.strictEqual(JWA.formDefaults(cfg, "nb").workspace.useDefaultSC, true);
  cfg.workspaceVolume.value.newPvc.spec.storageClassName = "fast";
  const ws = JWA.formDefaults(cfg, "nb").workspace;
  assert.deepStrictEqual([ws.useDefaultSC, ws.storageClass], [false, "fast"]);
  assert.strictEqual(JWA.buildBody(JWA.formDefaults(cfg, "nb"), cfg, "team").workspace.newPvc.spec.storageClassName, "fast");
});

test("VWA volume overview: facts, owner chips, pods mounted grouped into links (volume-details-page/overview)", () => {
  const pvc = { metadata: { name: "data", ownerReferences: [{ kind: "Notebook", name: "nb" }] },
                spec: { accessModes: ["ReadWriteOnce"], resources: { requests: { storage: "5Gi" } }, storageClassName: "fast" },
                status: { capacity: { storage: "8Gi" }, accessModes: ["ReadWriteMany"] } };
  assert.deepStrictEqual(VWA.overview(pvc), { accessModes: ["ReadWriteMany"], size: "8Gi", storageClass: "fast", volumeMode: "null",
                                              volumeName: "null", ownerRefs: ["Notebook: nb"] });
  assert.strictEqual(VWA.overview({ spec: { resources: { requests: { storage: "5Gi" } } } }).size, "5Gi");
  const pods = [
    { metadata: { namespace: "team", labels: { "notebook-name": "nb1" } } },
    { metadata: { namespace: "team", labels: { "serving.kubeflow.org/inferenceservice": "svc", component: "predictor" } } },
    { metadata: { namespace: "team", labels: { app: "other" } } },
    { metadata: { namespace: "team", labels: { "notebook-name": "nb2" } } }];
  assert.deepStrictEqual(VWA.podGroups(pods, "/x"), [
    { name: "Notebooks", links: [{ name: "nb1", url: "/x/jupyter/notebook/details/team/nb1/" }, { name: "nb2", url: "/x/jupyter/notebook/details/team/nb2/" }] },
    { name: "InferenceService", links: [{ name: "svc (predictor)", url: "/x/models/details/team/svc/" }] }]);
  assert.strictEqual(VWA.podsMountedMessage(""), "No pods are using this PVC.");
  assert.strictEqual(VWA.podsMountedMessage("boom"), "Failed to fetch mounted pods with error: boom");
});

test("VWA index page: every PVC name in name order with the reference status icons", () => {
  const pvcs = fixture("volumes", "pvcs").pvcs;
  checkTable(pvcs, VWA.columns(false));
  // the fixture predates the backend's {status, url} viewer object: both shapes are understood
  assert.deepStrictEqual(VWA.viewerState({ viewer: "ready" }), { status: "ready", url: null });
  assert.deepStrictEqual(VWA.viewerState({ viewer: { status: "ready", url: "/pvcviewers/ns/x/" } }), { status: "ready", url: "/pvcviewers/ns/x/" });
  assert.strictEqual(VWA.browseLabel({ viewer: { status: "uninitialized" } }), "Browse");
  assert.deepStrictEqual(VWA.newPvcBody("v1", "10", "ReadWriteOnce", ""), { name: "v1", size: "10Gi", mode: "ReadWriteOnce", class: "{empty}", type: "empty" });
  assert.deepStrictEqual(VWA.validate("ok-name", "5"), []);
  assert.strictEqual(VWA.validate("ok-name", "five").length, 1);
  // index-default.component.ts button states: in-use claims cannot be deleted, a claim waiting for its
  // first consumer may start a viewer, a requested viewer shows "waiting" and opens once ready
  const row = (phase, viewer, extra) => Object.assign({ name: "v", status: { phase }, viewer, notebooks: [] }, extra || {});
  assert.strictEqual(VWA.actionStates(row("ready", { status: "uninitialized" }, { notebooks: ["nb"] })).deleteAction, "unavailable");
  assert.strictEqual(VWA.actionStates(row("terminating", { status: "uninitialized" })).deleteAction, "terminating");
  assert.strictEqual(VWA.actionStates(row("waiting", { status: "uninitialized" })).openAction, "unavailable");
  const wffc = row("unavailable", { status: "uninitialized" });
  wffc.status.state = "WaitForFirstConsumer";
  assert.strictEqual(VWA.actionStates(wffc).openAction, "uninitialized");
  const w = new Set(["v"]);
  assert.deepStrictEqual(VWA.actionStates(row("ready", { status: "waiting" }), w),
                         { deleteAction: "ready", openAction: "waiting", closeAction: "ready", autoOpen: false });
  assert.strictEqual(VWA.actionStates(row("ready", { status: "ready", url: "/u" }), w).autoOpen, true);
  assert.strictEqual(w.has("v"), false);
  assert.strictEqual(VWA.actionStates(row("ready", { status: "terminating" })).closeAction, "waiting");
  assert.strictEqual(VWA.actionStates(row("ready", { status: "uninitialized" })).closeAction, "unavailable");
});

test("JWA index page: reference action states and optimistic rows", () => {
  const st = (phase) => JWA.actionStates({ status: { phase } });
  assert.deepStrictEqual(st("ready"), { deleteAction: "ready", connectAction: "ready", startStopAction: "uninitialized" });
  assert.deepStrictEqual(st("stopped"), { deleteAction: "ready", connectAction: "unavailable", startStopAction: "ready" });
  assert.deepStrictEqual(st("terminating"), { deleteAction: "terminating", connectAction: "unavailable", startStopAction: "unavailable" });
  assert.strictEqual(st("waiting").startStopAction, "uninitialized");
  const r = JWA.markPending({ name: "nb", status: { phase: "ready" } }, "stop");
  assert.deepStrictEqual([r.status.phase, r.status.message, r.connectAction], ["waiting", "Preparing to stop the Notebook Server.", "unavailable"]);
  assert.strictEqual(JWA.markPending({ status: { phase: "ready" } }, "delete").deleteAction, "terminating");
  assert.strictEqual(JWA.markPending({ status: { phase: "stopped" } }, "start").status.message, "Starting the Notebook Server.");
});

test("TWA index page: every TensorBoard name in name order with the reference status icons", () => {
  const tbs = fixture("tensorboards", "tensorboards").tensorboards;
  checkTable(tbs, TWA.columns(false));
  assert.strictEqual(TWA.logspath("pvc", "claim", "/logs/run1"), "pvc://claim/logs/run1");
  assert.strictEqual(TWA.logspath("object", "", " s3://b/run "), "s3://b/run");
  assert.deepStrictEqual(TWA.validate("tb", "object", "", "s3://bucket/x"), []);
  assert.strictEqual(TWA.validate("tb", "object", "", "/local").length, 1);
  assert.deepStrictEqual(TWA.validate("tb", "object", "", "s3://bucket/x", new Set(["tb"])), ["TensorBoard tb already exists"]);
  // index.component.ts processIncomingData: action states follow the phase; age split into value/tooltip
  const [ready, term, wait] = TWA.process([
    { name: "a", status: { phase: "ready" }, age: { uptime: "2 min", timestamp: "2024-01-01T00:00:00Z" } },
    { name: "b", status: { phase: "terminating" } }, { name: "c", status: { phase: "waiting" } }]);
  assert.deepStrictEqual([ready.connectAction, ready.deleteAction, ready.ageValue, ready.ageTooltip],
                         ["ready", "ready", "2 min", "2024-01-01T00:00:00Z"]);
  assert.deepStrictEqual([term.connectAction, term.deleteAction], ["unavailable", "terminating"]);
  assert.deepStrictEqual([wait.connectAction, wait.deleteAction], ["unavailable", "ready"]);
  const gone = TWA.markDeleting(ready);
  assert.deepStrictEqual([gone.status.phase, gone.deleteAction], ["terminating", "unavailable"]);
});

test("resource table: header click order, numeric sort, filter, escaping", () => {
  const cols = [{ title: "Name", value: (r) => r.name }, { title: "GPUs", value: (r) => r.gpus }];
  const rows = [{ name: "b", gpus: 8 }, { name: "a", gpus: 10 }, { name: "c", gpus: 2 }];
  assert.deepStrictEqual(kf.sortedRows({ columns: cols }, rows).map((r) => r.name), ["a", "b", "c"]);
  assert.deepStrictEqual(kf.sortedRows({ columns: cols }, rows, { sortCol: 1, sortDir: -1 }).map((r) => r.gpus), [10, 8, 2]);
  assert.deepStrictEqual(kf.sortedRows({ columns: cols }, rows, { filter: "C" }).map((r) => r.name), ["c"]);
  const html = kf.renderTable({ columns: [{ title: "Name", value: (r) => r.name }], actions: [{ name: "x", label: "X", enabled: () => false }] },
    [{ name: '<img src=x onerror="alert(1)">' }]);
  assert.ok(!html.includes("<img"), html);
  assert.ok(html.includes("disabled"));
  assert.ok(kf.renderTable({ columns: cols, empty: "Nothing here" }, []).includes("Nothing here"));
});

test("conditions table, logs viewer, quantities, name validator", () => {
  const ct = kf.conditionsTable([{ type: "Ready", status: "True", lastTransitionTime: "t1" },
                                 { type: "PodScheduled", status: "False", reason: "Unschedulable", message: "<b>no</b>" }]);
  assert.ok(ct.includes("check_circle") && ct.includes("warning") && ct.includes("Unschedulable") && !ct.includes("<b>"));
  assert.ok(kf.conditionsTable([]).includes("No conditions"));
  const logs = kf.renderLogs(["alpha", "beta <x>", "gamma"], "");
  assert.ok(logs.includes('<span class="ln">3</span> gamma') && logs.includes("beta &lt;x&gt;"));
  const filtered = kf.renderLogs(["alpha", "beta", "alphabet"], "alpha");
  assert.ok(filtered.includes('<span class="ln">3</span> alphabet') && !filtered.includes("beta<"));
  assert.strictEqual(kf.parseQuantity("1.5"), 1.5);
  assert.strictEqual(kf.parseQuantity("500m"), 0.5);
  assert.strictEqual(kf.parseQuantity("2Gi"), 2 * 1024 ** 3);
  assert.ok(isNaN(kf.parseQuantity("2 GB")));
  assert.strictEqual(kf.validators.name("nb-1"), "");
  assert.ok(kf.validators.name("-nb").length > 0);
  assert.ok(kf.validators.name("a".repeat(64)).includes("at most 63"));
  assert.strictEqual(kf.validators.limitAtLeastRequest("2Gi", "2048Mi", "Memory"), "");
});

test("resource table: filter chips (any column / column:value, AND-ed) and date / memory columns", () => {
  const nbs = fixture("jupyter", "notebooks").notebooks;
  const cols = JWA.columns(false);
  const terms = kf.parseFilter("Status:ready, rstudio,");
  assert.deepStrictEqual(terms, [{ column: "status", value: "ready" }, "rstudio"]);
  const names = (filter) => kf.sortedRows({ columns: cols }, nbs, { filter }).map((r) => r.name);
  assert.deepStrictEqual(names("terminating"), nbs.filter((n) => n.status.phase === "terminating").map((n) => n.name).sort());
  assert.deepStrictEqual(names("status:stopped"), nbs.filter((n) => n.status.phase === "stopped").map((n) => n.name).sort());
  // every chip must match: a name chip AND a phase chip
  const one = nbs.find((n) => n.status.phase === "ready");
  assert.deepStrictEqual(names(`${one.name}, status:ready`), [one.name]);
  assert.deepStrictEqual(names(`${one.name},status:stopped`), []);
  // Memory is a MemoryValue: "1073741824m" (a milli-byte quantity) shows as 1.0 Mi, "1Gi" as 1.0 Gi
  const html = kf.renderTable({ columns: cols }, nbs);
  const mem = column(html, "Memory");
  nbs.slice().sort((a, b) => a.name.localeCompare(b.name)).forEach((n, i) =>
    assert.strictEqual(mem[i], kf.formatBytes(kf.quantityToScalar(n.memory))));
  assert.ok(mem.includes("1.0 Mi") && mem.includes("1.0 Gi"), mem);
  // Created at / Last activity: relative time with the UTC time on hover; "-" when unset
  const created = column(html, "Created at");
  assert.ok(created.every((c) => /ago<\/span>$/.test(c) && c.includes("UTC: 20")), created[0]);
  assert.ok(column(html, "Last activity").includes("-"));
  // a date column filters on its words too ("... days ago" / "... years ago")
  assert.strictEqual(names("created at:ago").length, nbs.length);
  // sorting a date column sorts by time, a memory column by bytes
  const byAge = kf.sortedRows({ columns: cols }, nbs, { sortCol: cols.findIndex((c) => c.title === "Created at"), sortDir: 1 });
  assert.deepStrictEqual(byAge.map((r) => r.age), nbs.map((r) => r.age).sort());
  const byMem = kf.sortedRows({ columns: cols }, nbs, { sortCol: cols.findIndex((c) => c.title === "Memory"), sortDir: 1 });
  assert.strictEqual(byMem[0].memory, "1073741824m");
});

test("resource table paginator: 10 / 20 / 50 per page, range label, buttons", () => {
  const cols = [{ title: "Name", value: (r) => r.name }];
  const rows = Array.from({ length: 23 }, (_, i) => ({ name: `nb-${String(i).padStart(2, "0")}` }));
  assert.deepStrictEqual(kf.PAGE_SIZES, [10, 20, 50]);
  assert.deepStrictEqual(kf.paginate(23, 2, 10), { page: 2, size: 10, pages: 3, start: 20, end: 23, label: "21 – 23 of 23" });
  assert.strictEqual(kf.paginate(23, 9, 10).page, 2);       // clamped to the last page
  assert.strictEqual(kf.paginate(23, 0, 7).size, 50);       // unknown size -> default 50
  assert.strictEqual(kf.paginate(0, 0, 10).label, "0 of 0");
  const page1 = kf.renderTable({ columns: cols }, rows, { page: 1, pageSize: 10 });
  assert.deepStrictEqual(column(page1, "Name"), rows.slice(10, 20).map((r) => r.name));
  assert.ok(page1.includes("11 – 20 of 23") && page1.includes("data-cy-paginator"));
  assert.ok(!/data-page="prev" disabled/.test(page1) && !/data-page="next" disabled/.test(page1));
  const first = kf.renderTable({ columns: cols }, rows, { page: 0, pageSize: 20 });
  assert.ok(/data-page="prev" disabled/.test(first) && first.includes("1 – 20 of 23"));
  assert.ok(!kf.renderTable({ columns: cols }, rows.slice(0, 5)).includes("data-cy-paginator"));
});

test("quantities, bytes and relative time (resource-table utils, lib-date-time)", () => {
  assert.strictEqual(kf.quantityToScalar("500m"), 0.5);
  assert.strictEqual(kf.quantityToScalar("2Gi"), 2 * 2 ** 30);
  assert.strictEqual(kf.quantityToScalar("1.5k"), 1500);
  assert.strictEqual(kf.quantityToScalar("10"), 10);
  assert.strictEqual(kf.quantityToScalar(""), 0);
  assert.throws(() => kf.quantityToScalar("3 bananas"));
  assert.strictEqual(kf.formatBytes(512), "512 B");
  assert.strictEqual(kf.formatBytes(1536), "1.5 Ki");
  assert.strictEqual(kf.formatBytes(20 * 2 ** 30), "20.0 Gi");
  assert.strictEqual(kf.formatBytes(1023.99 * 2 ** 20), "1.0 Gi");  // rounds up into the next unit
  assert.strictEqual(kf.formatBytes(1.5e9, true), "1.5 GB");
  const now = Date.parse("2024-03-10T12:00:00Z");
  const ago = (ms) => kf.timeAgo(new Date(now - ms).toISOString(), now);
  const M = 60e3, H = 60 * M, D = 24 * H;
  assert.strictEqual(ago(10e3), "less than a minute ago");
  assert.strictEqual(ago(1 * M), "1 minute ago");
  assert.strictEqual(ago(44 * M), "44 minutes ago");
  assert.strictEqual(ago(50 * M), "1 hour ago");
  assert.strictEqual(ago(5 * H), "5 hours ago");
  assert.strictEqual(ago(30 * H), "1 day ago");
  assert.strictEqual(ago(12 * D), "12 days ago");
  assert.strictEqual(ago(40 * D), "1 month ago");
  assert.strictEqual(ago(200 * D), "7 months ago");
  assert.strictEqual(kf.timeAgo("2023-02-01T12:00:00Z", now), "1 year ago");
  assert.strictEqual(kf.timeAgo("2022-09-10T12:00:00Z", now), "over 1 year ago");
  assert.strictEqual(kf.timeAgo("2021-04-10T12:00:00Z", now), "3 years ago");
  assert.strictEqual(kf.timeAgo(new Date(now + 3 * H).toISOString(), now), "in 3 hours");
  assert.strictEqual(kf.timeAgo("", now), "-");
  assert.strictEqual(kf.dateTimeHtml(""), "-");
});

test("confirm dialogs: the reference texts, applying state, error kept in the dialog", () => {
  const d = JWA.dialogs.delete("nb1");
  assert.strictEqual(d.title, "Are you sure you want to delete this notebook server? nb1");
  assert.strictEqual(d.accept, "DELETE");
  assert.strictEqual(d.applying, "DELETING");
  assert.strictEqual(JWA.dialogs.stop("nb1").confirmColor, "primary");
  assert.strictEqual(VWA.dialogs.delete("v").message, "Warning: All data in this volume will be lost.");
  assert.strictEqual(VWA.dialogs.closeViewer("v").accept, "CLOSE");
  assert.strictEqual(TWA.dialogs.delete("t").title, "Are you sure you want to delete this Tensorboard : t ?");
  const idle = kf.renderConfirm(d, false);
  assert.ok(idle.includes('data-resp="accept" class="warn">DELETE</button>') && idle.includes(">CANCEL</button>"));
  const busy = kf.renderConfirm(d, true);
  assert.ok(!busy.includes('data-resp="accept"') && busy.includes("DELETING") && busy.includes("disabled"));
  const failed = kf.renderConfirm(Object.assign({}, d, { error: "<forbidden>" }), false);
  assert.ok(failed.includes("&lt;forbidden&gt;") && failed.includes('data-resp="accept"'));
});

test("JWA form-gpus: vendor list, 'not installed' tooltip, vendor-with-num (form-gpus.component.ts:25-77)", () => {
  const cfg = fixture("jupyter", "config").config;  // vendors NVIDIA + AMD, vendor "", num "none"
  const f = JWA.formDefaults(cfg, "nb");
  assert.deepStrictEqual(f.gpus, { num: "none", vendor: "" });
  // num "none": the vendor control is disabled, and no vendor is required
  assert.strictEqual(JWA.vendorDisabled(f.gpus), true);
  assert.strictEqual(JWA.vendorError(f.gpus), "");
  // /api/gpus reported only amd.com/gpu: NVIDIA keeps its option with the tooltip
  const installed = new Set(["amd.com/gpu"]);
  const [nv, amd] = JWA.gpuVendors(cfg);
  assert.strictEqual(JWA.vendorTooltip(nv, installed), "There are currently no NVIDIA GPUs in your cluster.");
  assert.strictEqual(JWA.vendorTooltip(amd, installed), "");
  const html = JWA.vendorOptions(cfg, f.gpus, installed);
  assert.ok(html.startsWith('<option value=""></option>'), html);  // no vendor chosen yet
  assert.ok(html.includes('value="nvidia.com/gpu" title="There are currently no NVIDIA GPUs in your cluster.">NVIDIA'));
  assert.ok(html.includes('value="amd.com/gpu" title="">AMD'));
  // a count without a vendor is the vendorNullName error, in validate() too
  const g = { num: "2", vendor: "" };
  assert.strictEqual(JWA.vendorDisabled(g), false);
  assert.strictEqual(JWA.vendorError(g), "You must also specify the GPU Vendor for the assigned GPUs");
  assert.ok(JWA.validate(Object.assign({}, f, { name: "nb", gpus: g })).includes("You must also specify the GPU Vendor for the assigned GPUs"));
  const ok = { num: "2", vendor: "amd.com/gpu" };
  assert.strictEqual(JWA.vendorError(ok), "");
  assert.ok(JWA.vendorOptions(cfg, ok, installed).includes('value="amd.com/gpu" title="" selected>AMD'));
  // nothing installed at all (CPU cluster): every vendor gets the tooltip
  assert.ok(JWA.vendorOptions(cfg, ok, new Set()).includes("There are currently no AMD GPUs in your cluster."));
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try { await fn(); console.log("ok -", name); } catch (e) { failed++; console.log("FAIL -", name, "\n", e && e.stack); }
  }
  if (failed) process.exit(1);
})();
