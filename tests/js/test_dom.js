// DOM-level tests of the JWA page (jupyter/static/index.html + assets/app.js + common kf.js) on the
// fake DOM of fakedom.js: the page boots against a scripted backend, then the table's action
// buttons and the spawner form are driven the way a user drives them (clicks, selects, typing) and
// the HTTP calls the page makes are asserted. Ports the behaviour of the reference's
// jupyter/frontend/src/app/pages/index/index-default (button wiring + confirm dialogs) and
// pages/form/form-new/form-gpus/form-gpus.component.ts (vendor select, tooltip, vendorWithNum).
// argv[2] = the reference crud-web-apps directory (its Cypress fixtures are the backend's data).
"use strict";
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const vm = require("vm");
const { Document, Node, choose, type } = require("./fakedom.js");

const WEB = path.join(__dirname, "../../kubeflow_rm_amd/webapps");
const FIX = process.argv[2];
const fixture = (name) => JSON.parse(fs.readFileSync(path.join(FIX, "jupyter/frontend/cypress/fixtures", name + ".json"), "utf8"));

// ---- browser globals -----------------------------------------------------------------------------------
global.window = global;
global.Node = Node;
global.document = new Document(fs.readFileSync(path.join(WEB, "jupyter/static/index.html"), "utf8"));
global.location = { search: "?ns=team" };
global.localStorage = { getItem: () => null, setItem: () => {} };
global.addEventListener = () => {};
global.parent = global;
global.postMessage = () => {};
const opened = [];
global.open = (url) => opened.push(url);
const realSetTimeout = setTimeout;
global.setTimeout = (fn, ms) => (ms > 100 ? 0 : realSetTimeout(fn, ms));  // no background polling
global.clearTimeout = () => {};

// ---- scripted backend ----------------------------------------------------------------------------------
const config = fixture("config").config;  // GPU vendors NVIDIA + AMD, no default vendor
const notebooks = fixture("notebooks").notebooks;
const calls = [];
const overrides = {};
global.fetch = async (url, opts) => {
  const method = (opts && opts.method) || "GET";
  const body = opts && opts.body ? JSON.parse(opts.body) : undefined;
  calls.push({ method, url, body });
  const key = `${method} ${url}`;
  let data = { success: true };
  if (overrides[key]) data = overrides[key];
  else if (url === "api/config") data = { success: true, config };
  else if (url === "api/namespaces") data = { success: true, namespaces: ["team"] };
  else if (url === "api/namespaces/team/notebooks" && method === "GET") data = { success: true, notebooks };
  else if (url === "api/namespaces/team/poddefaults") data = { success: true, poddefaults: [{ label: "add-gpu-env", desc: "GPU env" }] };
  else if (url === "api/namespaces/team/pvcs") data = { success: true, pvcs: [{ name: "data" }] };
  else if (url === "api/gpus") data = { success: true, vendors: ["amd.com/gpu"] };
  else if (url === "api/storageclasses") data = { success: true, storageClasses: ["standard", "fast-nvme"] };
  else if (url === "api/storageclasses/default") data = { success: true, defaultStorageClass: "standard" };
  const ok = data.success !== false;
  return { ok, status: ok ? 200 : 403, statusText: ok ? "OK" : "Forbidden", json: async () => data };
};

const settle = async (n = 10) => { for (let i = 0; i < n; i++) await new Promise((r) => setImmediate(r)); };
const $ = (id) => document.getElementById(id);
const lastCall = (method) => calls.filter((c) => c.method === method).slice(-1)[0];

vm.runInThisContext(fs.readFileSync(path.join(WEB, "crud_backend/static/kf.js"), "utf8"));
vm.runInThisContext(fs.readFileSync(path.join(WEB, "jupyter/static/assets/app.js"), "utf8"));

const tests = [];
const test = (name, fn) => tests.push([name, fn]);
const btn = (action, name) => document.querySelectorAll(`#notebooks button[data-action="${action}"]`)
  .find((b) => b.getAttribute("data-key").split("/").pop() === name) || null;
const nsOf = (r) => r.namespace || "team";
const byPhase = (phase) => notebooks.find((r) => r.status.phase === phase);

test("page boots: config, namespaces and the notebook table from the backend", async () => {
  await settle();
  assert.ok(calls.some((c) => c.url === "api/config"));
  const rows = document.querySelectorAll("#notebooks tbody tr");
  assert.strictEqual(rows.length, notebooks.length);
});

test("table: Stop on a ready notebook confirms, then PATCHes stopped=true and marks the row", async () => {
  const nb = byPhase("ready");
  btn("toggle", nb.name).click();
  const dlg = document.querySelector("dialog.confirm");
  assert.ok(dlg && dlg.open, "confirm dialog shown");
  assert.ok(dlg.textContent.includes(`Are you sure you want to stop this notebook server? ${nb.name}`));
  dlg.querySelector('button[data-resp="accept"]').click();
  await settle();
  const c = lastCall("PATCH");
  assert.deepStrictEqual([c.url, c.body], [`api/namespaces/${nsOf(nb)}/notebooks/${nb.name}`, { stopped: true }]);
  assert.strictEqual(document.querySelector("dialog.confirm"), null, "dialog closed after success");
});

test("table: a failing Stop keeps the dialog open with the backend's error", async () => {
  // another row whose toggle is an enabled "Stop" (the warning-phase notebook)
  const nb = byPhase("warning");
  assert.ok(btn("toggle", nb.name) && !btn("toggle", nb.name).disabled && btn("toggle", nb.name).textContent === "Stop");
  overrides[`PATCH api/namespaces/${nsOf(nb)}/notebooks/${nb.name}`] = { success: false, log: "forbidden: <stop>" };
  // re-render with fresh rows (the previous test marked its row pending)
  calls.length = 0;
  btn("toggle", nb.name).click();
  const dlg = document.querySelector("dialog.confirm");
  dlg.querySelector('button[data-resp="accept"]').click();
  await settle();
  const again = document.querySelector("dialog.confirm");
  assert.ok(again && again.textContent.includes("forbidden: <stop>"), "error shown in the dialog");
  again.querySelector('button[data-resp="cancel"]').click();
  await settle();
  assert.strictEqual(document.querySelector("dialog.confirm"), null);
  delete overrides[`PATCH api/namespaces/${nsOf(nb)}/notebooks/${nb.name}`];
});

test("table: Start on a stopped notebook PATCHes stopped=false without a dialog", async () => {
  const nb = byPhase("stopped");
  btn("toggle", nb.name).click();
  await settle();
  assert.strictEqual(document.querySelector("dialog.confirm"), null);
  const c = lastCall("PATCH");
  assert.deepStrictEqual([c.url, c.body], [`api/namespaces/${nsOf(nb)}/notebooks/${nb.name}`, { stopped: false }]);
});

test("table: Connect opens the notebook URL only when ready; Delete confirms then DELETEs", async () => {
  const ready = notebooks.find((r) => r.status.phase === "ready" && btn("connect", r.name) && !btn("connect", r.name).disabled);
  if (ready) {
    btn("connect", ready.name).click();
    assert.strictEqual(opened.pop(), `/notebook/${nsOf(ready)}/${ready.name}/`);
  }
  const stopped = byPhase("stopped");
  const cb = btn("connect", stopped.name);
  assert.ok(cb.disabled, "connect disabled for a stopped notebook");
  cb.click();
  assert.strictEqual(opened.length, 0);
  const victim = notebooks.find((r) => btn("delete", r.name) && !btn("delete", r.name).disabled);
  btn("delete", victim.name).click();
  const dlg = document.querySelector("dialog.confirm");
  assert.ok(dlg.textContent.includes(`Are you sure you want to delete this notebook server? ${victim.name}`));
  dlg.querySelector('button[data-resp="accept"]').click();
  await settle();
  assert.strictEqual(lastCall("DELETE").url, `api/namespaces/${nsOf(victim)}/notebooks/${victim.name}`);
});

test("spawner: GPU vendor select from the config, 'not installed' tooltip, disabled while count is none", async () => {
  $("new").click();
  await settle();
  assert.ok($("spawner").open, "spawner dialog open");
  assert.ok(calls.some((c) => c.url === "api/gpus"), "installed vendors fetched");
  const v = $("f-gpu-vendor");
  const opts = v.options.map((o) => [o.value, o.textContent, o.getAttribute("title")]);
  assert.deepStrictEqual(opts, [["", "", null],
    ["nvidia.com/gpu", "NVIDIA", "There are currently no NVIDIA GPUs in your cluster."],
    ["amd.com/gpu", "AMD", ""]]);
  assert.strictEqual($("f-gpus").value, "none");
  assert.ok(v.disabled, "vendor disabled while num is none");
  choose($("f-gpus"), "2");
  assert.ok(!$("f-gpu-vendor").disabled, "vendor enabled once a count is chosen");
});

test("spawner: a GPU count without a vendor is refused (vendorNullName), then the chosen vendor is POSTed", async () => {
  type($("f-name"), "my-nb");
  const posts = () => calls.filter((c) => c.method === "POST").length;
  const before = posts();
  $("f-submit").click();
  await settle();
  assert.strictEqual(posts(), before, "no POST while the vendor is missing");
  assert.ok($("f-error").textContent.includes("You must also specify the GPU Vendor for the assigned GPUs"), $("f-error").textContent);
  assert.ok($("f-gpu-vendor-err").textContent.includes("You must also specify the GPU Vendor"));
  choose($("f-gpu-vendor"), "amd.com/gpu");
  assert.strictEqual($("f-gpu-vendor-err").textContent, "");
  $("f-submit").click();
  await settle();
  const c = lastCall("POST");
  assert.strictEqual(c.url, "api/namespaces/team/notebooks");
  assert.strictEqual(c.body.name, "my-nb");
  assert.deepStrictEqual(c.body.gpus, { num: "2", vendor: "amd.com/gpu" });
  assert.strictEqual(c.body.workspace.newPvc.metadata.name, "{notebook-name}-workspace");
  assert.ok(!$("spawner").open, "spawner closed after a successful create");
  assert.ok(document.getElementById("kf-snack").textContent.includes("Notebook my-nb created"));
});

test("spawner: count back to none sends no vendor requirement", async () => {
  $("new").click();
  await settle();
  type($("f-name"), "cpu-nb");
  choose($("f-gpus"), "none");
  assert.ok($("f-gpu-vendor").disabled);
  $("f-submit").click();
  await settle();
  const c = lastCall("POST");
  assert.strictEqual(c.body.name, "cpu-nb");
  assert.deepStrictEqual(c.body.gpus, { num: "none" });
});

test("spawner: a Custom (Advanced) data volume is edited as YAML; a parse error blocks the POST", async () => {
  $("new").click();
  await settle();
  type($("f-name"), "yaml-nb");
  $("f-add-vol").click();
  const row = () => document.querySelector("#f-datavols .datavol");
  choose(row().querySelector(".dv-kind"), "custom");
  const ta = () => row().querySelector(".dv-yaml textarea");
  assert.ok(ta(), "YAML editor shown for the custom volume");
  assert.ok(ta().value.includes("name: yaml-nb-datavol-1"), ta().value);  // typeChanged dumps the current PVC
  assert.ok(row().querySelector(".dv-name").hidden && row().querySelector(".dv-size").hidden);
  const posts = () => calls.filter((c) => c.method === "POST").length;
  const text = (ind) => `metadata:\n  name: big\nspec:\n  resources:\n    requests:\n      storage: 100Gi\n${ind}accessModes: [ReadWriteOnce]`;
  type(ta(), text("   "));
  assert.ok(row().querySelector(".yaml-error").textContent.startsWith("bad indentation of a mapping entry (7:4)"),
    row().querySelector(".yaml-error").textContent);
  const before = posts();
  $("f-submit").click();
  await settle();
  assert.strictEqual(posts(), before, "no POST while the YAML does not parse");
  assert.ok($("f-error").textContent.includes("Data volume: bad indentation"), $("f-error").textContent);
  type(ta(), text("  "));
  assert.strictEqual(row().querySelector(".yaml-error").textContent, "");
  assert.strictEqual(row().querySelector(".gutter").textContent, "1\n2\n3\n4\n5\n6\n7");
  assert.ok(row().querySelector(".hl").innerHTML.includes('<span class="y-k">storage</span>'));
  $("f-submit").click();
  await settle();
  const c = lastCall("POST");
  assert.strictEqual(c.body.name, "yaml-nb");
  assert.deepStrictEqual(c.body.datavols[0].newPvc,
    { metadata: { name: "big" }, spec: { resources: { requests: { storage: "100Gi" } }, accessModes: ["ReadWriteOnce"] } });
});

test("spawner: the workspace volume's Custom (Advanced) type sends the edited PVC", async () => {
  $("new").click();
  await settle();
  type($("f-name"), "ws-nb");
  choose($("f-ws-kind"), "custom");
  assert.ok($("f-ws-fields").hidden && !$("f-ws-custom").hidden);
  const ta = $("f-ws-yaml").querySelector("textarea");
  assert.ok(ta.value.includes("storage: 20Gi"), ta.value);
  type(ta, ta.value.replace("20Gi", "64Gi"));
  $("f-submit").click();
  await settle();
  const c = lastCall("POST");
  assert.strictEqual(c.body.name, "ws-nb");
  assert.strictEqual(c.body.workspace.newPvc.spec.resources.requests.storage, "64Gi");
  choose($("f-ws-kind"), "empty");
  assert.ok(!$("f-ws-fields").hidden && $("f-ws-custom").hidden);
});

test("spawner: storage class — default ticked sends none, an explicit class is POSTed (storage-class component)", async () => {
  $("new").click();
  await settle();
  type($("f-name"), "sc-nb");
  assert.ok($("f-ws-sc-default").checked && $("f-ws-sc").disabled);
  assert.strictEqual($("f-ws-sc").value, "standard", "disabled select shows the default class");
  $("f-add-vol").click();
  const row = document.querySelector("#f-datavols .datavol");
  const cb = row.querySelector(".dv-sc-default");
  cb.checked = false;
  cb.dispatchEvent({ type: "change" });
  const sel = document.querySelector("#f-datavols .datavol .dv-sc");
  assert.ok(!sel.disabled);
  assert.deepStrictEqual(sel.options.map((o) => o.textContent), ["Empty storage class", "standard", "fast-nvme"]);
  choose(sel, "fast-nvme");
  $("f-submit").click();
  await settle();
  const c = lastCall("POST");
  assert.strictEqual(c.body.name, "sc-nb");
  assert.ok(!("storageClassName" in c.body.workspace.newPvc.spec));
  assert.strictEqual(c.body.datavols[0].newPvc.spec.storageClassName, "fast-nvme");
});

test("notebook overview: volumes by kind, configuration dialog with the PodDefault as YAML, env groups", async () => {
  const nb = byPhase("ready");
  const ns = nsOf(nb);
  const base = `api/namespaces/${ns}/notebooks/${nb.name}`;
  overrides[`GET ${base}`] = { success: true, notebook: {
    metadata: { name: nb.name, namespace: ns, labels: { "add-gpu-env": "true" }, annotations: {} },
    spec: { template: { spec: { containers: [{ name: nb.name, image: "img", env: [{ name: "A", value: "1" }], resources: {} }],
                                volumes: [{ name: "ws", persistentVolumeClaim: { claimName: "ws" } }, { name: "dshm", emptyDir: { medium: "Memory" } }] } } },
    status: { conditions: [] } } };
  overrides[`GET ${base}/pod`] = { success: true, pod: { metadata: { name: `${nb.name}-0`, labels: { "notebook-name": nb.name } },
    spec: { containers: [{ name: nb.name, env: [{ name: "A", value: "1" }, { name: "HIP_VISIBLE_DEVICES", value: "0" }] }] } } };
  overrides[`GET api/namespaces/${ns}/poddefaults`] = { success: true, poddefaults: [{ label: "add-gpu-env", desc: "GPU env",
    metadata: { name: "gpu-env" }, spec: { desc: "GPU env", selector: { matchLabels: { "add-gpu-env": "true" } }, env: [{ name: "HIP_VISIBLE_DEVICES", value: "0" }] } }] };
  document.querySelectorAll("#notebooks a.name").find((a) => a.getAttribute("data-open").split("/").pop() === nb.name).click();
  await settle();
  await new Promise((r) => realSetTimeout(r, 5));
  const body = $("kf-details").querySelector(".tab-body");
  assert.ok(body.textContent.includes("Shared memory enabled"), body.textContent.slice(0, 200));
  assert.ok(body.querySelector(`a.vol-link[href="/volumes/volume/details/${ns}/ws"]`), "PVC links to the volumes app");
  assert.ok(body.textContent.includes("Memory-backed Volumes"));
  assert.ok(body.textContent.includes("gpu-env (Configuration)") && body.textContent.includes("HIP_VISIBLE_DEVICES: 0"));
  body.querySelector("button.config-link").click();
  const info = document.querySelector("dialog.info");
  assert.ok(info && info.open && info.textContent.includes("gpu-env:"));
  assert.ok(info.querySelector(".hl").textContent.includes("Description: GPU env") && !info.querySelector(".hl").textContent.includes("name: gpu-env"));
  info.querySelector('button[data-resp="close"]').click();
  assert.strictEqual(document.querySelector("dialog.info"), null);
  $("kf-details").querySelector("button[data-close]").click();
  for (const k of [`GET ${base}`, `GET ${base}/pod`, `GET api/namespaces/${ns}/poddefaults`]) delete overrides[k];
});

test("notebook page YAML tab: Notebook / Pod select over a read-only editor (notebook-page/yaml)", async () => {
  const nb = byPhase("ready");
  const base = `api/namespaces/${nsOf(nb)}/notebooks/${nb.name}`;
  overrides[`GET ${base}`] = { success: true, notebook: { apiVersion: "kubeflow.org/v1", kind: "Notebook", metadata: { name: nb.name } } };
  overrides[`GET ${base}/pod`] = { success: true, pod: { kind: "Pod", metadata: { name: `${nb.name}-0` } } };
  const link = document.querySelectorAll("#notebooks a.name").find((a) => a.getAttribute("data-open").split("/").pop() === nb.name);
  link.click();
  await settle();
  const dlg = $("kf-details");
  assert.ok(dlg && dlg.open, "details open");
  dlg.querySelectorAll("nav.tabs button[data-tab]").find((b) => b.textContent === "YAML").click();
  await settle();
  await new Promise((r) => realSetTimeout(r, 5));
  await settle();
  const body = dlg.querySelector(".tab-body");
  assert.ok(body.textContent.includes("Show the full YAML of the"));
  assert.ok(body.querySelector(".yaml-editor.ro") && !body.querySelector("textarea"), "read-only editor");
  assert.ok(body.querySelector(".hl").textContent.includes("kind: Notebook"), body.querySelector(".hl").textContent);
  choose(body.querySelector("select.yaml-which"), "pod");
  assert.ok(body.querySelector(".hl").textContent.includes(`name: ${nb.name}-0`));
  choose(body.querySelector("select.yaml-which"), "notebook");
  assert.ok(body.querySelector(".hl").textContent.includes("kind: Notebook"));
  dlg.querySelector("button[data-close]").click();
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try { await fn(); console.log("ok -", name); } catch (e) { failed++; console.log("FAIL -", name, "\n", e && e.stack); }
  }
  process.exit(failed ? 1 : 0);
})();
